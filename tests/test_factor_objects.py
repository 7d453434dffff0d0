"""Factorization objects (models/factor.py): factor once, solve many; against
numpy, on the host target (single process).  The distributed path of the same
objects runs in dist_worker.case_factor_objects."""
import numpy as np
import pytest

import slate_d35_amd as s
from helpers import rnd


@pytest.mark.parametrize("method", ["tntpiv", "ppiv", "nopiv"])
def test_lu_factor_solve_many(method):
    n, nb = 150, 32
    a = rnd(n, n, np.float64, 1) + (n * np.eye(n) if method == "nopiv" else 0)
    F = s.LUFactor(s.from_numpy(a, nb=nb), method=method)
    for seed in (2, 3):
        b = rnd(n, 3, np.float64, seed)
        B = s.from_numpy(b, nb=nb)
        F.solve(B)
        np.testing.assert_allclose(a @ s.to_numpy(B), b, atol=1e-10 * n)
    if method != "nopiv":
        B = s.from_numpy(rnd(n, 2, np.float64, 4), nb=nb)
        b = s.to_numpy(B)
        F.solve(B, trans=s.Op.Trans)
        np.testing.assert_allclose(a.T @ s.to_numpy(B), b, atol=1e-10 * n)
    rc = F.rcond()
    exact = 1.0 / (np.linalg.norm(a, 1) * np.linalg.norm(np.linalg.inv(a), 1))
    assert exact / 10 <= rc <= exact * 10


def test_cholesky_factor():
    n, nb = 130, 32
    g = rnd(n, n, np.float64, 5)
    a = g @ g.T + n * np.eye(n)
    F = s.CholeskyFactor(s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb)))
    b = rnd(n, 2, np.float64, 6)
    B = s.from_numpy(b, nb=nb)
    F.solve(B)
    np.testing.assert_allclose(a @ s.to_numpy(B), b, atol=1e-10)
    assert F.rcond() > 0


def test_qr_factor_least_squares():
    m, n, nb = 200, 90, 32
    a = rnd(m, n, np.float64, 7)
    b = rnd(m, 2, np.float64, 8)
    F = s.QRFactor(s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    F.solve_ls(B)
    x = s.to_numpy(B)[:n]
    np.testing.assert_allclose(x, np.linalg.lstsq(a, b, rcond=None)[0], atol=1e-10)


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_mixed_lu_factor_refines_to_working_precision(dtype):
    n, nb = 160, 32
    a = rnd(n, n, dtype, 9) + 4 * np.eye(n)
    A = s.from_numpy(a, nb=nb)
    M = s.MixedLUFactor(A)
    for seed in (10, 11):
        b = rnd(n, 2, dtype, seed)
        X, it = M.solve(s.from_numpy(b, nb=nb))
        assert 0 <= it < 30
        x = s.to_numpy(X)
        r = np.linalg.norm(b - a @ x, np.inf) / (np.linalg.norm(a, np.inf) * np.linalg.norm(x, np.inf))
        assert r < 10 * np.finfo(np.float64).eps * np.sqrt(n)
    # the original matrix is untouched (the factor lives in a fp32 copy)
    np.testing.assert_array_equal(s.to_numpy(A), a)
