"""Factorization objects: factor once, solve many times.

The reference exposes this as the simplified API's ``lu_factor`` /
``lu_solve_using_factor`` / ``chol_solve_using_factor`` pairs
(include/slate/simplified_api.hh) and, for mixed precision, re-factors on
every ``gesv_mixed`` call (src/gesv_mixed.cc).  Here the factors, pivots,
the norm needed for condition estimates and (for the mixed-precision solver)
the low-precision copy live in one object, so a service answering many
right-hand sides against one matrix pays for the O(n^3) factorization once:

    F = LUFactor(A, method="tntpiv", target="d")     # A is overwritten by L\\U
    F.solve(B)                                        # B := A^{-1} B, O(n^2 nrhs)
    F.rcond()                                         # 1-norm estimate, no refactor

    M = MixedLUFactor(A, target="d")                  # fp32 LU of a copy; A kept
    X, iters = M.solve(B)                             # fp64 accuracy by refinement

Every method runs on the distributed matrices of the grid the operand lives
on (collective over its ranks), on the device when ``target="d"``.
"""
from __future__ import annotations

import numpy as np

from .. import _slate
from .._core import Matrix, Norm, Op, Side, Uplo, Diag, TriangularMatrix, empty_like, target_of
from . import aux, blas3, cholesky, lu, qr

__all__ = ["LUFactor", "CholeskyFactor", "QRFactor", "MixedLUFactor"]

_LOW = {np.dtype(np.float64): np.float32, np.dtype(np.complex128): np.complex64}


def _dtype_of(A):
    name = type(A).__name__
    return {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}[name[-1]]


def _like(A, dtype, target):
    """Matrix of A's shape, tiles and grid in another precision."""
    B = Matrix(A.m, A.n, A.nb, dtype, A.grid, mb=A.mb)
    B.insertLocalTiles(target_of(target) if target is not None else _slate.Target.Host)
    return B


class LUFactor:
    """A = P L U, in place in A (reference getrf / getrf_tntpiv / getrf_nopiv)."""

    def __init__(self, A, method="tntpiv", target=None, **kw):
        self.A, self.target, self.kw = A, target, kw
        self.anorm1 = aux.norm(Norm.One, A, target=target)   # before A is overwritten
        self.method = method
        if method == "nopiv":
            self.info = lu.getrf_nopiv(A, target=target, **kw)
            self.pivots = None
        else:
            fn = lu.getrf_tntpiv if method == "tntpiv" else lu.getrf
            self.info, self.pivots = fn(A, target=target, **kw)
        if self.info:
            raise np.linalg.LinAlgError(f"LUFactor: U({self.info},{self.info}) is exactly zero")

    def solve(self, B, trans=None):
        """op(A) X = B, X overwriting B."""
        if self.pivots is None:
            lu.getrs_nopiv(self.A, B, target=self.target, **self.kw)
        else:
            lu.getrs(self.A, self.pivots, B, target=self.target, trans=trans, **self.kw)
        return B

    def inverse(self, out=None):
        """A^{-1} (in place over the factors, or into `out`)."""
        if self.pivots is None:
            raise NotImplementedError("inverse needs a pivoted factorization")
        return lu.getri(self.A, self.pivots, out, target=self.target, **self.kw)

    def rcond(self):
        """Reciprocal 1-norm condition number estimate (reference gecondest)."""
        return lu.gecondest(Norm.One, self.A, self.anorm1, target=self.target)


class CholeskyFactor:
    """A = L L^H of a Hermitian positive definite matrix, in place."""

    def __init__(self, A, target=None, **kw):
        self.A, self.target, self.kw = A, target, kw
        self.anorm1 = aux.norm(Norm.One, A, target=target)
        self.info = cholesky.potrf(A, target=target, **kw)
        if self.info:
            raise np.linalg.LinAlgError(f"CholeskyFactor: leading minor {self.info} is not positive definite")

    def solve(self, B):
        cholesky.potrs(self.A, B, target=self.target, **self.kw)
        return B

    def inverse(self):
        """A^{-1} in place over the factor (reference potri)."""
        cholesky.potri(self.A, target=self.target, **self.kw)
        return self.A

    def rcond(self):
        return cholesky.pocondest(Norm.One, self.A, self.anorm1, target=self.target)


class QRFactor:
    """A = Q R (Householder, compact WY T factors), in place; least squares."""

    def __init__(self, A, target=None, **kw):
        self.A, self.target, self.kw = A, target, kw
        self.T = qr.geqrf(A, target=target, **kw)

    def apply_q(self, C, side=Side.Left, op=Op.NoTrans):
        """C := op(Q) C or C op(Q) (reference unmqr)."""
        qr.unmqr(side, op, self.A, self.T, C, target=self.target, **self.kw)
        return C

    def solve_ls(self, B):
        """min ||A X - B|| for m >= n: B := Q^H B, then R X = B(0:n) -- the
        solution is the first n rows of B (reference gels_qr)."""
        self.apply_q(B, Side.Left, Op.ConjTrans)
        n = self.A.n
        R = TriangularMatrix(Uplo.Upper, Diag.NonUnit, self.A.slice(0, n - 1, 0, n - 1))
        Bt = B if B.m == n else B.slice(0, n - 1, 0, B.n - 1)
        blas3.trsm(Side.Left, 1.0, R, Bt, target=self.target)
        return B


class MixedLUFactor:
    """Mixed precision: the LU of a low-precision copy (fp32 / complex64),
    factored ONCE; every solve refines in the working precision against the
    original A (kept untouched): x += A_lo^{-1} (b - A x) until the reference
    stopping test ||r|| <= ||x|| ||A||_inf eps sqrt(n) (src/gesv_mixed.cc).
    Falls back to a working-precision LU when refinement does not converge."""

    def __init__(self, A, method="tntpiv", target=None, max_iterations=30, **kw):
        self.A, self.target, self.kw = A, target, kw
        self.itermax = max_iterations
        dt = np.dtype(_dtype_of(A))
        if dt not in _LOW:
            raise TypeError("MixedLUFactor: fp64 / complex128 matrices only")
        self.dt = dt
        self.anorm = aux.norm(Norm.Inf, A, target=target)
        self.lo = _like(A, _LOW[dt], target)
        aux.copy(A, self.lo, target=target)
        self.F = LUFactor(self.lo, method=method, target=target, **kw)
        self.hi = None   # working-precision fallback factor, made on demand

    def solve(self, B, X=None):
        """Returns (X, iterations); iterations < 0: refinement did not
        converge and the working-precision fallback produced X."""
        tg = self.target
        if X is None:
            X = empty_like(B, target=tg)
        n = self.A.n
        eps = np.finfo(self.dt).eps
        cte = self.anorm * eps * np.sqrt(n)
        R = empty_like(B, target=tg)
        C = empty_like(B, target=tg)
        Rlo = _like(B, _LOW[self.dt], tg)
        # x0 = A_lo^{-1} b
        aux.copy(B, Rlo, target=tg)
        self.F.solve(Rlo)
        aux.copy(Rlo, X, target=tg)
        for it in range(1, self.itermax + 1):
            aux.copy(B, R, target=tg)
            blas3.gemm(-1.0, self.A, X, 1.0, R, target=tg)          # r = b - A x
            # per right-hand side, as the reference (gesv_mixed.cc:209-212):
            # every column must meet ||r_j|| <= ||x_j|| ||A|| eps sqrt(n)
            rn = np.asarray(aux.colNorms(Norm.Max, R, target=tg))
            xn = np.asarray(aux.colNorms(Norm.Max, X, target=tg))
            if np.all(rn <= xn * cte):
                return X, it - 1
            aux.copy(R, Rlo, target=tg)
            self.F.solve(Rlo)
            aux.copy(Rlo, C, target=tg)
            aux.add(1.0, C, 1.0, X, target=tg)                      # x += c
        # fallback: working-precision LU of a copy of A
        if self.hi is None:
            Ah = empty_like(self.A, target=tg)
            aux.copy(self.A, Ah, target=tg)
            self.hi = LUFactor(Ah, method="ppiv", target=tg, **self.kw)
        aux.copy(B, X, target=tg)
        self.hi.solve(X)
        return X, -self.itermax
