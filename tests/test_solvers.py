"""Condition estimators and GMRES-IR (reference test/test_gecondest.cc,
test_pocondest.cc, test_trcondest.cc, test_gesv.cc --method gmres)."""
import numpy as np
import pytest

import slate_d35_amd as s
from helpers import DTYPES, rnd, relerr, butterfly_dense as _butterfly


def _ill(n, dt, seed, cond=1e4):
    rng = np.random.default_rng(seed)
    u, _ = np.linalg.qr(rng.standard_normal((n, n)))
    v, _ = np.linalg.qr(rng.standard_normal((n, n)))
    sv = np.logspace(0, -np.log10(cond), n)
    return (u * sv) @ v.T


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("norm", ["one", "inf"])
def test_gecondest(dtype, norm):
    n = 150
    a = (_ill(n, dtype, 3) + (1j * _ill(n, dtype, 4) if np.iscomplexobj(np.zeros(1, dtype)) else 0)).astype(dtype)
    nk = s.Norm.One if norm == "one" else s.Norm.Inf
    npn = 1 if norm == "one" else np.inf
    A = s.from_numpy(a, nb=32)
    anorm = s.norm(nk, A)
    info, _ = s.getrf(A)
    assert info == 0
    rc = s.gecondest(nk, A, anorm)
    ref = 1.0 / (np.linalg.norm(a, npn) * np.linalg.norm(np.linalg.inv(a.astype(np.complex128)), npn))
    assert ref * 0.999 <= rc <= 10 * ref, (rc, ref)


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_pocondest(dtype):
    n = 120
    b = _ill(n, dtype, 5, 1e3).astype(dtype)
    a = b @ b.conj().T + 1e-6 * np.eye(n)
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a.astype(dtype), nb=32))
    anorm = s.norm(s.Norm.One, A)
    assert s.potrf(A) == 0
    rc = s.pocondest(s.Norm.One, A, anorm)
    ref = 1.0 / np.linalg.cond(a, 1)
    assert ref * 0.999 <= rc <= 10 * ref, (rc, ref)


@pytest.mark.parametrize("uplo", ["L", "U"])
def test_trcondest(uplo):
    n = 100
    t = rnd(n, n, np.float64, 6) + 4 * np.eye(n)
    t = np.tril(t) if uplo == "L" else np.triu(t)
    u = s.Uplo.Lower if uplo == "L" else s.Uplo.Upper
    T = s.TriangularMatrix(u, s.Diag.NonUnit, s.from_numpy(t, nb=32))
    for nk, npn in [(s.Norm.One, 1), (s.Norm.Inf, np.inf)]:
        rc = s.trcondest(nk, T)
        ref = 1.0 / np.linalg.cond(t, npn)
        assert ref * 0.999 <= rc <= 10 * ref, (rc, ref)


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_gesv_mixed_gmres(dtype):
    n = 180
    a = (_ill(n, dtype, 7, 1e5)).astype(dtype)
    if np.iscomplexobj(a):
        a = a + 1j * _ill(n, dtype, 8, 1e2)
    b = rnd(n, 1, dtype, 9)
    A, B = s.from_numpy(a, nb=32), s.from_numpy(b, nb=32)
    X = s.from_numpy(np.zeros_like(b), nb=32)
    info, _, it = s.gesv_mixed_gmres(A, B, X)
    assert info == 0 and it >= 0
    x = s.to_numpy(X)
    assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 1e-14


def test_posv_mixed_gmres():
    n = 160
    c = _ill(n, np.float64, 10, 1e3)
    a = c @ c.T + 1e-3 * np.eye(n)
    b = rnd(n, 1, np.float64, 11)
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=32))
    B, X = s.from_numpy(b, nb=32), s.from_numpy(np.zeros_like(b), nb=32)
    info, it = s.posv_mixed_gmres(A, B, X)
    assert info == 0 and it >= 0
    x = s.to_numpy(X)
    assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 1e-14


@pytest.mark.parametrize("dtype", DTYPES)
def test_gesv_rbt(dtype):
    n = 130
    a = rnd(n, n, dtype, 21)
    # a matrix whose leading entries make no-pivot LU unstable without the RBT
    a[0, 0] = 1e-10
    b = rnd(n, 2, dtype, 22)
    A, B = s.from_numpy(a, nb=32), s.from_numpy(b, nb=32)
    X = s.from_numpy(np.zeros_like(b), nb=32)
    info, it = s.gesv_rbt(A, B, X)
    assert info == 0
    x = s.to_numpy(X)
    eps = np.finfo(np.float32 if dtype in (np.float32, np.complex64) else np.float64).eps
    assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 100 * n * eps


def test_gerbt_depths():
    n = 97
    a = rnd(n, n, np.float64, 23)
    for depth in (1, 2, 3):
        A = s.from_numpy(a, nb=16)
        s.gerbt(A, depth)
        ap = s.to_numpy(A)
        # a similarity-free two-sided transform preserves rank / nonsingularity
        assert abs(np.linalg.slogdet(ap)[1]) < np.inf
        assert not np.allclose(ap, a)


def test_getri_out_of_place():
    n = 90
    a = rnd(n, n, np.float64, 24) + n * np.eye(n)
    A = s.from_numpy(a, nb=32)
    info, piv = s.getrf(A)
    B = s.from_numpy(np.zeros((n, n)), nb=32)
    s.getri(A, piv, B)
    assert relerr(s.to_numpy(B) @ a, np.eye(n)) < 1e-13


def _lu_residual(a, f, piv, nb):
    m, n = a.shape
    k = min(m, n)
    L = np.tril(f[:, :k], -1) + np.eye(m, k)
    U = np.triu(f[:k, :])
    pa = a.copy()
    for j, p_ in enumerate(kk * nb + ti * nb + off for kk, pv in enumerate(piv) for (ti, off) in pv):
        pa[[j, p_]] = pa[[p_, j]]
    return relerr(L @ U, pa), np.abs(L).max()


@pytest.mark.parametrize("thresh", [1.0, 0.5, 0.1])
def test_getrf_pivot_threshold(thresh):
    """Option::PivotThreshold (reference src/getrf.cc:39): the diagonal stays
    pivot while |a_jj| >= threshold * column max, so |L| <= 1 / threshold and
    fewer rows move as the threshold drops."""
    n, nb = 120, 32
    a = rnd(n, n, np.float64, 61) + 1.5 * np.eye(n)

    def moved(piv):
        return sum(1 for blk in piv for j, (ti, off) in enumerate(blk) if (ti, off) != (0, j))
    A = s.from_numpy(a, nb=nb)
    info, piv = s.getrf(A, pivot_threshold=thresh)
    err, lmax = _lu_residual(a, s.to_numpy(A), piv, nb)
    assert info == 0 and err < 1e-12
    assert lmax <= 1.0 / thresh + 1e-12
    if thresh < 1.0:
        A1 = s.from_numpy(a, nb=nb)
        _, piv1 = s.getrf(A1)
        assert moved(piv) < moved(piv1), (moved(piv), moved(piv1))


def test_getrf_pivot_threshold_invalid():
    A = s.from_numpy(rnd(40, 40, np.float64, 62), nb=16)
    with pytest.raises(Exception):
        s.getrf(A, pivot_threshold=1.5)


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_gerbt_matches_dense_butterflies(depth):
    """gerbt applies the O(n^2 d) butterfly levels: equal to U^T A V with the
    dense butterflies (seeds of gerbt's defaults)."""
    m, n, nb = 75, 61, 16
    a = rnd(m, n, np.float64, 25)
    A = s.from_numpy(a, nb=nb)
    s.gerbt(A, depth, 1, 2)
    U, V = _butterfly(m, depth, 1), _butterfly(n, depth, 2)
    assert relerr(s.to_numpy(A), U.T @ a @ V) < 1e-14


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
@pytest.mark.parametrize("nrhs", [1, 3])
def test_mixed_escalate_gmres(dtype, nrhs):
    """Option::EscalateGmres: on a matrix too ill-conditioned for classical
    fp32 refinement (kappa ~ 1e8: kappa eps_32 > 1, refinement
    stalls or diverges), gesv_mixed / posv_mixed switch to GMRES-IR with the SAME fp32
    factors instead of the fp64 refactorization.  Default (reference
    semantics): classical refinement, then the fallback (iter < 0)."""
    n = 192
    a = _ill(n, dtype, 51, 1e8).astype(dtype)
    b = rnd(n, nrhs, dtype, 52)
    res = {}
    for esc in (False, True):
        A, B = s.from_numpy(a, nb=32), s.from_numpy(b, nb=32)
        X = s.from_numpy(np.zeros_like(b), nb=32)
        info, _, it = s.gesv_mixed(A, B, X, escalate_gmres=esc, max_iterations=20)
        x = s.to_numpy(X)
        assert info == 0
        assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 1e-14
        res[esc] = it
    assert res[False] < 0, res          # classical refinement gave up -> fp64 fallback
    assert res[True] > 0, res           # escalation converged on the fp32 factors
    # Hermitian positive definite: posv_mixed
    c = _ill(n, dtype, 53, 1e4)
    h = (c @ c.conj().T).astype(dtype)
    for esc in (False, True):
        H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=32))
        B, X = s.from_numpy(b, nb=32), s.from_numpy(np.zeros_like(b), nb=32)
        info, it = s.posv_mixed(H, B, X, escalate_gmres=esc, max_iterations=20)
        x = s.to_numpy(X)
        assert info == 0
        assert np.linalg.norm(h @ x - b) / (np.linalg.norm(h) * np.linalg.norm(x)) < 1e-14
        assert (it > 0) if esc else (it < 0), (esc, it)
