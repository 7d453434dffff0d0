"""Level-3 BLAS (reference src/gemm*.cc, hemm*.cc, symm.cc, herk.cc, syrk.cc,
her2k.cc, syr2k.cc, trmm.cc, trsm*.cc)."""
from ._wrap import call

__all__ = ["gbmm", "hbmm", "tbsm", "gemm", "gemmA", "gemmC", "hemm", "symm", "herk", "syrk", "her2k", "syr2k",
           "trmm", "trsm", "multiply", "triangular_multiply", "triangular_solve",
           "rank_k_update", "rank_2k_update"]


def gemm(alpha, A, B, beta, C, target=None, **kw):
    """C = alpha A B + beta C (SUMMA gemmC, or gemmA for a single block column)."""
    call("gemm", C, alpha, A, B, beta, C, target=target, **kw)


def gemmA(alpha, A, B, beta, C, target=None, **kw):
    call("gemmA", C, alpha, A, B, beta, C, target=target, **kw)


def gemmC(alpha, A, B, beta, C, target=None, **kw):
    call("gemmC", C, alpha, A, B, beta, C, target=target, **kw)


def hemm(side, alpha, A, B, beta, C, target=None, **kw):
    call("hemm", C, side, alpha, A, B, beta, C, target=target, **kw)


def symm(side, alpha, A, B, beta, C, target=None, **kw):
    call("symm", C, side, alpha, A, B, beta, C, target=target, **kw)


def herk(alpha, A, beta, C, target=None, **kw):
    call("herk", C, alpha, A, beta, C, target=target, **kw)


def syrk(alpha, A, beta, C, target=None, **kw):
    call("syrk", C, alpha, A, beta, C, target=target, **kw)


def her2k(alpha, A, B, beta, C, target=None, **kw):
    call("her2k", C, alpha, A, B, beta, C, target=target, **kw)


def syr2k(alpha, A, B, beta, C, target=None, **kw):
    call("syr2k", C, alpha, A, B, beta, C, target=target, **kw)


def trmm(side, alpha, A, B, target=None, **kw):
    call("trmm", B, side, alpha, A, B, target=target, **kw)


def trsm(side, alpha, A, B, target=None, **kw):
    call("trsm", B, side, alpha, A, B, target=target, **kw)


# simplified API names (reference include/slate/simplified_api.hh)
def multiply(alpha, A, B, beta, C, **kw):
    name = type(A).__name__
    from .._core import Side
    if name.startswith("HermitianMatrix"):
        return hemm(Side.Left, alpha, A, B, beta, C, **kw)
    if name.startswith("SymmetricMatrix"):
        return symm(Side.Left, alpha, A, B, beta, C, **kw)
    if type(B).__name__.startswith("HermitianMatrix"):
        return hemm(Side.Right, alpha, B, A, beta, C, **kw)
    if type(B).__name__.startswith("SymmetricMatrix"):
        return symm(Side.Right, alpha, B, A, beta, C, **kw)
    return gemm(alpha, A, B, beta, C, **kw)


def triangular_multiply(alpha, A, B, **kw):
    from .._core import Side
    if type(A).__name__.startswith("TriangularMatrix"):
        return trmm(Side.Left, alpha, A, B, **kw)
    return trmm(Side.Right, alpha, B, A, **kw)


def triangular_solve(alpha, A, B, **kw):
    from .._core import Side
    if type(A).__name__.startswith("TriangularMatrix"):
        return trsm(Side.Left, alpha, A, B, **kw)
    return trsm(Side.Right, alpha, B, A, **kw)


def rank_k_update(alpha, A, beta, C, **kw):
    if type(C).__name__.startswith("HermitianMatrix"):
        return herk(alpha, A, beta, C, **kw)
    return syrk(alpha, A, beta, C, **kw)


def rank_2k_update(alpha, A, B, beta, C, **kw):
    if type(C).__name__.startswith("HermitianMatrix"):
        return her2k(alpha, A, B, beta, C, **kw)
    return syr2k(alpha, A, B, beta, C, **kw)


def gbmm(alpha, A, B, beta, C, target=None, **kw):
    """C = alpha A B + beta C with A a BandMatrix (reference src/gbmm.cc)."""
    call("gbmm", A, alpha, A, B, beta, C, target=target, **kw)


def hbmm(side, alpha, A, B, beta, C, target=None, **kw):
    """C = alpha A B + beta C (or B A) with A a HermitianBandMatrix (src/hbmm.cc)."""
    call("hbmm", A, side, alpha, A, B, beta, C, target=target, **kw)


def tbsm(side, alpha, A, B, target=None, pivots=None, **kw):
    """Solve op(A) X = alpha B with A a TriangularBandMatrix (src/tbsm.cc).
    pivots (per tile: [(tile offset, row offset), ...], as gbtrf / getrf
    return them): the row interchanges of tile k are applied to B(k:, :)
    before tile k's solve on a forward sweep, after it on a backward sweep
    (reference src/tbsmPivots.cc)."""
    if pivots is not None:
        return call("tbsm_pivots", A, side, alpha, A, [list(map(tuple, p)) for p in pivots], B, target=target, **kw)
    call("tbsm", A, side, alpha, A, B, target=target, **kw)
