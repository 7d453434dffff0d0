"""Cholesky family (reference src/potrf.cc, potrs.cc, posv.cc, potri.cc,
posv_mixed.cc, posv_mixed_gmres.cc, pocondest.cc)."""
from ._wrap import call

__all__ = ["potrf", "potrs", "posv", "potri", "posv_mixed", "posv_mixed_gmres", "pocondest",
           "chol_factor", "chol_solve", "chol_solve_using_factor", "chol_inverse_using_factor",
           "chol_rcondest_using_factor"]


def potrf(A, target=None, **kw):
    """A = L L^H (or U^H U); returns info (0 on success)."""
    return call("potrf", A, A, target=target, **kw)


def potrs(A, B, target=None, **kw):
    call("potrs", A, A, B, target=target, **kw)


def posv(A, B, target=None, **kw):
    return call("posv", A, A, B, target=target, **kw)


def potri(A, target=None, **kw):
    return call("potri", A, A, target=target, **kw)


def posv_mixed(A, B, X, target=None, **kw):
    """fp32 Cholesky + fp64 iterative refinement; returns (info, iterations)."""
    return call("posv_mixed", A, A, B, X, target=target, **kw)


def posv_mixed_gmres(A, B, X, target=None, **kw):
    return call("posv_mixed_gmres", A, A, B, X, target=target, **kw)


def pocondest(norm, A, anorm, target=None, **kw):
    return call("pocondest", A, norm, A, anorm, target=target, **kw)


chol_factor = potrf
chol_solve = posv
chol_solve_using_factor = potrs
chol_inverse_using_factor = potri
chol_rcondest_using_factor = pocondest
