"""Eigenvalue / SVD drivers (reference src/heev.cc, hegv.cc, hegst.cc,
he2hb.cc, hb2st.cc, sterf.cc, steqr2.cc, stedc*.cc, svd.cc, ge2tb.cc,
tb2bd.cc, bdsqr.cc)."""
from ._wrap import call

__all__ = ["heev", "hegv", "hegst", "svd", "svd_vals", "eig", "eig_vals", "he2hb", "hb2st", "sterf",
           "steqr", "stedc", "ge2tb", "tb2bd", "bdsqr"]


def heev(A, Z=None, target=None, **kw):
    """Eigenvalues (and vectors into Z if given) of a Hermitian matrix."""
    return call("heev", A, A, Z, target=target, **kw)


def hegv(itype, A, B, Z=None, target=None, **kw):
    return call("hegv", A, itype, A, B, Z, target=target, **kw)


def hegst(itype, A, B, target=None, **kw):
    return call("hegst", A, itype, A, B, target=target, **kw)


def svd(A, U=None, VT=None, target=None, **kw):
    return call("svd", A, A, U, VT, target=target, **kw)


def svd_vals(A, target=None, **kw):
    return svd(A, None, None, target=target, **kw)


def eig(A, Z, **kw):
    return heev(A, Z, **kw)


def eig_vals(A, **kw):
    return heev(A, None, **kw)


def he2hb(A, target=None, **kw):
    return call("he2hb", A, A, target=target, **kw)


def hb2st(A, target=None, **kw):
    return call("hb2st", A, A, target=target, **kw)


def sterf(d, e, **kw):
    from .. import _slate
    return _slate.sterf(list(d), list(e))


def steqr(d, e, Z=None, **kw):
    from .. import _slate
    return _slate.steqr(list(d), list(e), Z is not None)


def stedc(d, e, **kw):
    from .. import _slate
    return _slate.stedc(list(d), list(e))


def ge2tb(A, target=None, **kw):
    return call("ge2tb", A, A, target=target, **kw)


def tb2bd(A, target=None, **kw):
    return call("tb2bd", A, A, target=target, **kw)


def bdsqr(d, e, **kw):
    from .. import _slate
    return _slate.bdsqr(list(d), list(e))
