"""Test-matrix generation (reference matgen/generate_matrix_*.cc).

Values come from a counter-based generator keyed by (global i, global j,
seed), so a matrix is identical for any process grid and target (the
reference's matgen/random.cc:53-110 uses Philox-2x64 for the same property).
The generator itself is native (csrc/src/matgen.cc + kernels/matgen.hip,
formulas in kernels/matgen_entry.hh); this module exposes it to Python:

    sigma, cond = generate_matrix("svd_geo", A, cond=1e6)   # distributed A in place
    a = generate("kms", 100)                                 # numpy, 1 x 1 host

plus `random_matrix`, a pure-numpy mirror of the counter hash that the tests
use to build reference inputs bit-identical to the native fill.
"""
from __future__ import annotations

import numpy as np

__all__ = ["random_matrix", "spd_matrix", "diag_dominant_matrix", "generate", "generate_matrix", "usage", "KINDS"]

KINDS = ["zeros", "ones", "identity", "ij", "jordan", "jordanT", "chebspec", "circul", "fiedler", "gfpp", "kms",
         "orthog", "riemann", "ris", "zielkeNS", "rand", "rands", "randn", "randb", "randr",
         "diag", "svd", "poev", "spd", "heev", "syev", "geev"]

_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0x632BE59BD9B4E019)
_M3 = np.uint64(0xD1B54A32D192ED03)
_M4 = np.uint64(0x94D049BB133111EB)


def _hash(i, j, seed):
    # SplitMix64 finaliser of an (i, j, seed) key: matgen_entry.hh unit()
    with np.errstate(over="ignore"):
        x = (np.asarray(i, dtype=np.uint64) * _M1
             ^ (np.asarray(j, dtype=np.uint64) + _M2) * _M3
             ^ np.uint64(seed) * _M4)
        x = x ^ (x >> np.uint64(30)); x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27)); x = x * _M4
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)


def _sample(kind, i, j, seed):
    u = _hash(i, j, seed)
    if kind == "rand":
        return u
    if kind == "randb":
        return np.where(u < 0.5, 0.0, 1.0)
    if kind == "randr":
        return np.where(u < 0.5, -1.0, 1.0)
    if kind == "randn":
        v = _hash(i, j, seed ^ 0x5851F42D4C957F2D)
        return np.sqrt(-2.0 * np.log(1.0 - u)) * np.cos(6.283185307179586 * v)
    return 2.0 * u - 1.0


def random_matrix(m, n, seed=42, dtype=np.float64, kind="rands"):
    """numpy mirror of the native random kinds (identical values)."""
    i, j = np.meshgrid(np.arange(m, dtype=np.uint64), np.arange(n, dtype=np.uint64), indexing="ij")
    a = _sample(kind, i, j, seed)
    if np.issubdtype(np.dtype(dtype), np.complexfloating):
        a = a + 1j * _sample(kind, i, j, seed + 7919)
    return a.astype(dtype)


def spd_matrix(n, seed=42, dtype=np.float64):
    """Hermitian positive definite: Hermitian rands + n*I (native kind 'spd' of the fast fill)."""
    a = random_matrix(n, n, seed, dtype)
    up = np.triu(a, 1)  # element (i, j) hashes (min, max); imaginary part negated above the diagonal
    h = up.T + up.conj() + np.diag(np.real(np.diag(a)))
    return (h + n * np.eye(n)).astype(dtype)


def diag_dominant_matrix(n, seed=42, dtype=np.float64):
    a = random_matrix(n, n, seed, dtype)
    a += n * np.eye(n, dtype=dtype)
    return a


def usage() -> str:
    from .. import _slate
    return _slate.generate_matrix_usage()


def generate_matrix(kind, A, seed=42, cond=None, condD=None, sigma=None, target=None):
    """Fill distributed matrix A (Matrix, or Hermitian/Symmetric/Triangular/
    Trapezoid view) with test matrix `kind` (see usage()).  Returns
    (Sigma, cond_actual): singular values / eigenvalues when known."""
    from .._core import native, opts
    nan = float("nan")
    c = nan if cond is None else float(cond)
    cd = nan if condD is None else float(condD)
    if type(A).__name__.split("_")[0] in ("HermitianMatrix", "SymmetricMatrix", "TriangularMatrix", "TrapezoidMatrix"):
        S, ca = native("matgen_tz", A)(kind, A, int(seed), c, cd, opts(target))
    else:
        S, ca = native("matgen", A)(kind, A, int(seed), c, cd, list(sigma) if sigma is not None else [],
                                    opts(target))
    return np.asarray(S), ca


def generate(kind, m, n=None, seed=42, dtype=np.float64, cond=None, condD=None, nb=256):
    """Generate an m x n test matrix as a numpy array (1 x 1 host grid)."""
    from .._core import Matrix, to_numpy
    from .. import _slate
    n = m if n is None else n
    A = Matrix(m, n, nb=nb, dtype=dtype, grid=_slate.Grid.self())
    A.insertLocalTiles(_slate.Target.HostTask)
    generate_matrix(kind, A, seed=seed, cond=cond, condD=condD, target="h")
    return to_numpy(A)
