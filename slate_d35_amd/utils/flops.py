"""LAWN-41 flop counts (reference docs/latex/flops.py:300-422)."""

__all__ = ["gemm_flops", "potrf_flops", "getrf_flops", "geqrf_flops", "gesv_flops", "trsm_flops",
           "herk_flops", "potrs_flops", "getrs_flops"]


def gemm_flops(m, n, k):
    return 2.0 * m * n * k


def potrf_flops(n):
    return n ** 3 / 3.0 + n ** 2 / 2.0 + n / 6.0


def getrf_flops(m, n=None):
    n = m if n is None else n
    if m == n:
        return 2.0 * n ** 3 / 3.0 - n ** 2 / 2.0 + 5.0 * n / 6.0
    if m > n:
        return m * n ** 2 - n ** 3 / 3.0 - n ** 2 / 2.0 + 5.0 * n / 6.0
    return n * m ** 2 - m ** 3 / 3.0 - m ** 2 / 2.0 + 5.0 * m / 6.0


def geqrf_flops(m, n=None):
    n = m if n is None else n
    if m == n:
        return 4.0 * n ** 3 / 3.0 + 2.0 * n ** 2 + 14.0 * n / 3.0
    if m > n:
        return 2.0 * m * n ** 2 - 2.0 * n ** 3 / 3.0 + m * n + n ** 2 + 14.0 * n / 3.0
    return 2.0 * n * m ** 2 - 2.0 * m ** 3 / 3.0 + 3.0 * m * n - m ** 2 + 14.0 * m / 3.0


def trsm_flops(m, n, left=True):
    return (n * m ** 2) if left else (m * n ** 2)


def herk_flops(n, k):
    return float(k) * n * (n + 1)


def potrs_flops(n, nrhs):
    return 2.0 * n ** 2 * nrhs


def getrs_flops(n, nrhs):
    return 2.0 * n ** 2 * nrhs


def gesv_flops(n, nrhs):
    return getrf_flops(n) + getrs_flops(n, nrhs)
