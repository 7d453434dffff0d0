"""Eigenvalue / SVD drivers (reference src/heev.cc, hegv.cc, hegst.cc,
he2hb.cc, hb2st.cc, sterf.cc, steqr2.cc, stedc*.cc, svd.cc, ge2tb.cc,
tb2bd.cc, bdsqr.cc)."""
from ._wrap import call

__all__ = ["heev", "hegv", "hegst", "svd", "svd_vals", "eig", "eig_vals", "he2hb", "hb2st", "sterf",
           "steqr", "stedc", "ge2tb", "tb2bd", "bdsqr"]


def heev(A, Z=None, target=None, **kw):
    """Eigenvalues (ascending numpy array; vectors into Z if given) of a
    Hermitian matrix.  method_eig="dc" (divide and conquer, default) or "qr"."""
    import numpy as np
    return np.asarray(call("heev", A, A, Z, target=target, **kw))


def hegv(itype, A, B, Z=None, target=None, **kw):
    """Generalized Hermitian-definite eigenproblem (itype 1: A x = l B x,
    2: A B x = l x, 3: B A x = l x).  B is overwritten by its Cholesky factor."""
    import numpy as np
    return np.asarray(call("hegv", A, itype, A, B, Z, target=target, **kw))


def hegst(itype, A, B, target=None, **kw):
    return call("hegst", A, itype, A, B, target=target, **kw)


def svd(A, U=None, VT=None, target=None, **kw):
    """Singular values (descending numpy array); thin U (m x k) and VT
    (k x n), k = min(m, n), filled when given."""
    import numpy as np
    return np.asarray(call("svd", A, A, U, VT, target=target, **kw))


def svd_vals(A, target=None, **kw):
    return svd(A, None, None, target=target, **kw)


def eig(A, Z, **kw):
    return heev(A, Z, **kw)


def eig_vals(A, **kw):
    return heev(A, None, **kw)


def he2hb(A, target=None, **kw):
    return call("he2hb", A, A, target=target, **kw)


def hb2st(a, kd):
    """Band (dense numpy, Hermitian, bandwidth kd) -> (d, e) of the tridiagonal."""
    import numpy as np
    from .._core import native
    return native("hb2st", np.asarray(a).dtype)(np.asarray(a), kd)


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


def tb2bd(a, kd):
    """Upper band (dense numpy, bandwidth kd) -> (d, e) of the bidiagonal."""
    import numpy as np
    from .._core import native
    return native("tb2bd", np.asarray(a).dtype)(np.asarray(a), kd)


def bdsqr(d, e, **kw):
    from .. import _slate
    return _slate.bdsqr(list(d), list(e))
