"""Auxiliary routines and norms (reference src/add.cc, copy.cc, scale.cc,
scale_row_col.cc, set.cc, set_lambdas.cc, redistribute.cc, norm.cc, colNorms.cc)."""
from .. import _slate
from .._core import suffix_of, opts
from ._wrap import call

__all__ = ["add", "tzadd", "copy", "scale", "scale_row_col", "set", "set_lambda", "redistribute",
           "norm", "colNorms", "print_matrix", "print_to_string"]


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


def print_to_string(label, A, target=None, **kw):
    """What slate::print writes on rank 0 (MATLAB-style block; '' elsewhere).
    Keywords: print_verbose (0-4, default 2), print_edge_items (16),
    print_width (10), print_precision (4)."""
    return call("print", A, label, A, target=target, **kw)


def print_matrix(label, A, target=None, **kw):
    """Collective print of a distributed matrix (reference slate::print)."""
    out = print_to_string(label, A, target=target, **kw)
    if out:
        print(out, end="", flush=True)
