"""LU family (reference src/getrf*.cc, getrs*.cc, gesv*.cc, getri*.cc,
gecondest.cc, trtri.cc, trtrm.cc, trcondest.cc)."""
from .. import _slate
from ._wrap import call

__all__ = ["getrf", "getrf_nopiv", "getrf_tntpiv", "getrs", "getrs_nopiv", "gesv", "gesv_nopiv",
           "gesv_mixed", "gesv_mixed_gmres", "gesv_rbt", "gerbt", "getri", "gecondest", "trtri", "trtrm",
           "trcondest", "lu_factor", "lu_solve", "lu_solve_using_factor", "lu_inverse_using_factor",
           "lu_factor_nopiv", "lu_solve_nopiv", "lu_solve_using_factor_nopiv", "lu_rcondest_using_factor",
           "triangular_rcondest", "gbtrf", "gbtrs", "gbsv", "pbtrf", "pbtrs", "pbsv", "hetrf", "hetrs", "hesv",
           "indefinite_factor", "indefinite_solve", "indefinite_solve_using_factor", "sysv", "hetrf_aasen",
           "hetrs_aasen", "hesv_aasen"]


def getrf(A, target=None, **kw):
    """LU with partial pivoting; returns (info, pivots) where pivots is a list
    of lists of (tile_index, offset) as the reference's Pivots."""
    return call("getrf", A, A, target=target, **kw)


def getrf_nopiv(A, target=None, **kw):
    return call("getrf_nopiv", A, A, target=target, **kw)


def getrf_tntpiv(A, target=None, **kw):
    """Communication-avoiding LU (tournament pivoting); returns (info, pivots)."""
    return call("getrf_tntpiv", A, A, target=target, **kw)


def getrs(A, pivots, B, target=None, trans=None, **kw):
    """op(A) X = B with the getrf factors (trans: Op.NoTrans / Trans / ConjTrans)."""
    if trans is not None and int(trans) != int(_slate.Op.NoTrans):
        call("getrs_op", A, trans, A, pivots, B, target=target, **kw)
        return
    call("getrs", A, A, pivots, B, target=target, **kw)


def getrs_nopiv(A, B, target=None, **kw):
    call("getrs_nopiv", A, A, B, target=target, **kw)


def gesv(A, B, target=None, **kw):
    """Returns (info, pivots)."""
    return call("gesv", A, A, B, target=target, **kw)


def gesv_nopiv(A, B, target=None, **kw):
    return call("gesv_nopiv", A, A, B, target=target, **kw)


def gesv_mixed(A, B, X, target=None, **kw):
    """fp32 LU + fp64 iterative refinement; returns (info, pivots, iterations)."""
    return call("gesv_mixed", A, A, B, X, target=target, **kw)


def gesv_mixed_gmres(A, B, X, target=None, **kw):
    return call("gesv_mixed_gmres", A, A, B, X, target=target, **kw)


def gesv_rbt(A, B, X, target=None, **kw):
    """Random-butterfly LU without pivoting + refinement; returns (info, iterations)."""
    return call("gesv_rbt", A, A, B, X, target=target, **kw)


def getri(A, pivots, B=None, target=None, **kw):
    """Inverse from the LU factors: in place, or out of place into B."""
    if B is not None:
        return call("getri_oop", A, A, pivots, B, target=target, **kw)
    return call("getri", A, A, pivots, target=target, **kw)


def gerbt(A, depth=2, seed_u=0x5eed0001, seed_v=0x5eed0002, target=None, **kw):
    """A := U^T A V with random butterflies of the given depth."""
    return call("gerbt", A, A, depth, seed_u, seed_v, target=target, **kw)


def gecondest(norm, A, anorm, target=None, **kw):
    return call("gecondest", A, norm, A, anorm, target=target, **kw)


def trtri(A, target=None, **kw):
    return call("trtri", A, A, target=target, **kw)


def trtrm(A, target=None, **kw):
    return call("trtrm", A, A, target=target, **kw)


def trcondest(norm, A, target=None, **kw):
    return call("trcondest", A, norm, A, target=target, **kw)


def gbtrf(A, target=None, **kw):
    return call("gbtrf", A, A, target=target, **kw)


def gbtrs(A, pivots, B, target=None, **kw):
    return call("gbtrs", A, A, pivots, B, target=target, **kw)


def gbsv(A, B, target=None, **kw):
    return call("gbsv", A, A, B, target=target, **kw)


def pbtrf(A, target=None, **kw):
    return call("pbtrf", A, A, target=target, **kw)


def pbtrs(A, B, target=None, **kw):
    return call("pbtrs", A, A, B, target=target, **kw)


def pbsv(A, B, target=None, **kw):
    return call("pbsv", A, A, B, target=target, **kw)


def hetrf(A, target=None, **kw):
    return call("hetrf", A, A, target=target, **kw)


def hetrs(A, factors, B, target=None, **kw):
    return call("hetrs", A, A, factors, B, target=target, **kw)


def hesv(A, B, target=None, **kw):
    return call("hesv", A, A, B, target=target, **kw)


def hetrf_aasen(A, T, target=None, **kw):
    """Aasen P A P^T = L T L^H (A Hermitian, Lower); T: a BandMatrix(nb, nb, ...)
    of A's size that receives the block-tridiagonal factor (band-LU factored).
    Returns (info, pivots, pivots2)."""
    return call("hetrf_aasen", A, A, T, target=target, **kw)


def hetrs_aasen(A, pivots, T, pivots2, B, target=None, **kw):
    return call("hetrs_aasen", A, A, pivots, T, pivots2, B, target=target, **kw)


def hesv_aasen(A, T, B, target=None, **kw):
    """Solve with Aasen's factorization; returns (info, pivots, pivots2)."""
    return call("hesv_aasen", A, A, T, B, target=target, **kw)


lu_factor = getrf
lu_solve = gesv
lu_solve_using_factor = getrs
lu_inverse_using_factor = getri
lu_factor_nopiv = getrf_nopiv
lu_solve_nopiv = gesv_nopiv
lu_solve_using_factor_nopiv = getrs_nopiv
lu_rcondest_using_factor = gecondest
triangular_rcondest = trcondest
indefinite_factor = hetrf
indefinite_solve = hesv
indefinite_solve_using_factor = hetrs


def sysv(A, B, target=None, **kw):
    """Real symmetric indefinite solve (A a SymmetricMatrix of a real type);
    returns (info, ipiv)."""
    return call("sysv", A, A, B, target=target, **kw)
