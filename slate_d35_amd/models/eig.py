"""Eigenvalue / SVD drivers (reference src/heev.cc, hegv.cc, hegst.cc,
he2hb.cc, hb2st.cc, sterf.cc, steqr2.cc, stedc*.cc, svd.cc, ge2tb.cc,
tb2bd.cc, bdsqr.cc)."""
from ._wrap import call

__all__ = ["heev", "hegv", "hegst", "svd", "svd_vals", "gesvd", "eig", "eig_vals", "he2hb", "hb2st", "sterf",
           "steqr", "stedc", "ge2tb", "tb2bd", "bdsqr", "syev", "sygv", "hb2st_band", "unmtr_hb2st",
           "unmtr_he2hb", "tb2bd_band", "unmbr_tb2bd", "unmbr_ge2tb", "steqr2", "stedc_matrix", "bdsqr_matrix"]


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


def gesvd(A, U=None, VT=None, target=None, **kw):
    """Compatibility name of svd (reference slate.hh gesvd)."""
    return svd(A, U, VT, target=target, **kw)


def syev(A, Z=None, target=None, **kw):
    """Real symmetric eigenproblem (A a SymmetricMatrix of a real type)."""
    import numpy as np
    return np.asarray(call("syev", A, A, Z, target=target, **kw))


def sygv(itype, A, B, Z=None, target=None, **kw):
    import numpy as np
    return np.asarray(call("sygv", A, itype, A, B, Z, target=target, **kw))


# ---- stage-level API on distributed matrices (reference slate.hh:1050-1334)
def hb2st_band(A, target=None, **kw):
    """HermitianBandMatrix -> (d, e, V): the real tridiagonal and the
    bulge-chasing reflectors (apply with unmtr_hb2st)."""
    return call("hb2st_band", A, A, target=target, **kw)


def unmtr_hb2st(side, op, V, C, target=None, **kw):
    return call("unmtr_hb2st", C, side, op, V, C, target=target, **kw)


def unmtr_he2hb(side, op, A, Ts, C, target=None, **kw):
    return call("unmtr_he2hb", C, side, op, A, Ts, C, target=target, **kw)


def tb2bd_band(A, target=None, **kw):
    """Upper TriangularBandMatrix -> (d, e, U, V) of A = U B V^H."""
    return call("tb2bd_band", A, A, target=target, **kw)


def unmbr_tb2bd(side, op, V, C, target=None, **kw):
    return call("unmbr_tb2bd", C, side, op, V, C, target=target, **kw)


def unmbr_ge2tb(side, op, A, Ts, C, target=None, **kw):
    return call("unmbr_ge2tb", C, side, op, A, Ts, C, target=target, **kw)


def steqr2(jobz, d, e, Z, target=None, **kw):
    """Tridiagonal QL with Z := Z * eigenvectors (jobz = Job.Vec)."""
    import numpy as np
    return np.asarray(call("steqr2", Z, jobz, list(d), list(e), Z, target=target, **kw))


def stedc_matrix(d, e, Q, target=None, **kw):
    """Tridiagonal divide and conquer into a distributed Q."""
    import numpy as np
    return np.asarray(call("stedc_mat", Q, list(d), list(e), Q, target=target, **kw))


def bdsqr_matrix(jobu, jobvt, d, e, U=None, VT=None, target=None, **kw):
    import numpy as np
    key = U if U is not None else VT
    return np.asarray(call("bdsqr_mat", key, jobu, jobvt, list(d), list(e), U, VT, target=target, **kw))
