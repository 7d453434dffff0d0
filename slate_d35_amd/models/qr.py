"""QR / LQ / least squares (reference src/geqrf.cc, unmqr.cc, gelqf.cc,
unmlq.cc, gels*.cc, cholqr.cc)."""
from ._wrap import call

__all__ = ["geqrf", "unmqr", "gelqf", "unmlq", "gels", "cholqr", "qr_factor", "qr_multiply_by_q",
           "lq_factor", "lq_multiply_by_q", "least_squares_solve", "gels_qr", "gels_cholqr"]


def geqrf(A, target=None, **kw):
    """Householder QR; returns the T factors (list of matrices)."""
    return call("geqrf", A, A, target=target, **kw)


def unmqr(side, op, A, T, C, target=None, **kw):
    call("unmqr", A, side, op, A, T, C, target=target, **kw)


def gelqf(A, target=None, **kw):
    return call("gelqf", A, A, target=target, **kw)


def unmlq(side, op, A, T, C, target=None, **kw):
    call("unmlq", A, side, op, A, T, C, target=target, **kw)


def gels(A, BX, target=None, **kw):
    return call("gels", A, A, BX, target=target, **kw)


def cholqr(A, R, target=None, **kw):
    return call("cholqr", A, A, R, target=target, **kw)


def gels_qr(A, BX, target=None, **kw):
    return call("gels_qr", A, A, BX, target=target, **kw)


def gels_cholqr(A, R, BX, target=None, **kw):
    """Least squares via CholeskyQR (m >= n): A := Q, R (n x n) upper."""
    return call("gels_cholqr", A, A, R, BX, target=target, **kw)


qr_factor = geqrf
qr_multiply_by_q = unmqr
lq_factor = gelqf
lq_multiply_by_q = unmlq
least_squares_solve = gels
