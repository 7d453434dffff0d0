"""Auxiliary routines and norms (reference src/add.cc, copy.cc, scale.cc,
scale_row_col.cc, set.cc, set_lambdas.cc, redistribute.cc, norm.cc, colNorms.cc)."""
from .. import _slate
from .._core import suffix_of, opts
from ._wrap import call

__all__ = ["add", "tzadd", "copy", "scale", "scale_row_col", "set", "set_lambda", "redistribute",
           "norm", "colNorms"]


def add(alpha, A, beta, B, target=None, **kw):
    n = type(B).__name__
    if n.startswith(("TrapezoidMatrix", "TriangularMatrix", "SymmetricMatrix", "HermitianMatrix")):
        return call("tzadd", B, alpha, A, beta, B, target=target, **kw)
    call("add", B, alpha, A, beta, B, target=target, **kw)


def tzadd(alpha, A, beta, B, target=None, **kw):
    call("tzadd", B, alpha, A, beta, B, target=target, **kw)


def copy(A, B, target=None, **kw):
    sa, sb = suffix_of(A), suffix_of(B)
    if sa == sb:
        return call("copy", B, A, B, target=target, **kw)
    fn = getattr(_slate, f"copy_{sa}2{sb}")
    return fn(A, B, opts(target, **kw))


def scale(numer, denom, A, target=None, **kw):
    call("scale", A, numer, denom, A, target=target, **kw)


def scale_row_col(equed, R, C, A, target=None, **kw):
    call("scale_row_col", A, equed, list(R), list(C), A, target=target, **kw)


def set(offdiag, diag, A, target=None, **kw):  # noqa: A001 (reference name)
    call("set", A, offdiag, diag, A, target=target, **kw)


def set_lambda(fn, A, target=None, **kw):
    call("set_lambda", A, fn, A, target=target, **kw)


def redistribute(A, B, target=None, **kw):
    call("redistribute", B, A, B, target=target, **kw)


def norm(kind, A, target=None, **kw):
    return call("norm", A, kind, A, target=target, **kw)


def colNorms(kind, A, target=None, **kw):
    return call("colNorms", A, kind, A, target=target, **kw)
