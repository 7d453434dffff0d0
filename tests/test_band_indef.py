"""Band and Hermitian-indefinite drivers (reference test/test_gbsv.cc,
test_pbsv.cc, test_gbmm.cc, test_hbmm.cc, test_tbsm.cc, test_hesv.cc)."""
import numpy as np
import pytest

import slate_d35_amd as s
from helpers import DTYPES, rnd, relerr


def tol(dt):
    return 1e-3 if dt in (np.float32, np.complex64) else 1e-11


def band(a, kl, ku):
    return np.tril(np.triu(a, -kl), ku)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("kl,ku", [(2, 3), (0, 4), (7, 1), (20, 20)])
def test_gbsv(dt, kl, ku):
    n, nb = 120, 32
    a = band(rnd(n, n, dt, 1), kl, ku) + (kl + ku + 2) * np.eye(n, dtype=dt)
    b = rnd(n, 3, dt, 2)
    A = s.BandMatrix(kl, ku, s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    info, piv = s.gbsv(A, B)
    assert info == 0
    assert relerr(a @ s.to_numpy(B), b) < 100 * tol(dt)
    # solve again with the factors
    B2 = s.from_numpy(b, nb=nb)
    s.gbtrs(A, piv, B2)
    assert relerr(a @ s.to_numpy(B2), b) < 100 * tol(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("uplo", ["L", "U"])
def test_pbsv(dt, uplo):
    n, nb, kd = 100, 32, 5
    c = band(rnd(n, n, dt, 3), kd, kd)
    a = (c + c.conj().T) / 2 + (2 * kd + 2) * np.eye(n)
    a = band(a, kd, kd).astype(dt)
    b = rnd(n, 2, dt, 4)
    u = s.Uplo.Lower if uplo == "L" else s.Uplo.Upper
    A = s.HermitianBandMatrix(u, kd, s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    assert s.pbsv(A, B) == 0
    assert relerr(a @ s.to_numpy(B), b) < 100 * tol(dt)


@pytest.mark.parametrize("dt", [np.float64, np.complex128])
def test_gbmm_hbmm_tbsm(dt):
    n, nb, kl, ku = 90, 32, 4, 6
    a = rnd(n, n, dt, 5)
    b = rnd(n, 20, dt, 6)
    c = rnd(n, 20, dt, 7)
    ab = band(a, kl, ku)
    # gbmm ignores entries outside the band even if the storage holds them
    A = s.BandMatrix(kl, ku, s.from_numpy(a, nb=nb))
    B, C = s.from_numpy(b, nb=nb), s.from_numpy(c, nb=nb)
    s.gbmm(2.0, A, B, 0.5, C)
    assert relerr(s.to_numpy(C), 2.0 * ab @ b + 0.5 * c) < tol(dt)
    h = (a + a.conj().T) / 2
    hb = band(h, kl, kl)
    H = s.HermitianBandMatrix(s.Uplo.Lower, kl, s.from_numpy(np.tril(h), nb=nb))
    C = s.from_numpy(c, nb=nb)
    s.hbmm(s.Side.Left, 1.0, H, B, 0.0, C)
    assert relerr(s.to_numpy(C), hb @ b) < tol(dt)
    t = np.tril(band(a, kl, 0)) + 4 * np.eye(n)
    T = s.TriangularBandMatrix(s.Uplo.Lower, s.Diag.NonUnit, kl, s.from_numpy(t, nb=nb))
    X = s.from_numpy(b, nb=nb)
    s.tbsm(s.Side.Left, 1.0, T, X)
    assert relerr(t @ s.to_numpy(X), b) < tol(dt)


def _tbsm_pivots_ref(t, b, piv, nb, lower, alpha):
    """numpy rendering of the reference's pivoted band solve
    (src/tbsmPivots.cc): forward sweep (lower) swapping tile k's rows before
    its solve, backward sweep (upper) swapping after it."""
    n = t.shape[0]
    x = alpha * b.copy()
    nt = -(-n // nb)

    def swap(k, forward):
        seq = [(k * nb + i, (k + ti) * nb + off) for i, (ti, off) in enumerate(piv[k])]
        for r, p in (seq if forward else reversed(seq)):
            x[[r, p]] = x[[p, r]]

    ks = range(nt) if lower else range(nt - 1, -1, -1)
    for k in ks:
        r0, r1 = k * nb, min(n, (k + 1) * nb)
        if lower:
            swap(k, True)
            x[r0:r1] = np.linalg.solve(t[r0:r1, r0:r1], x[r0:r1])
            x[r1:] -= t[r1:, r0:r1] @ x[r0:r1]
        else:
            x[r0:r1] -= t[r0:r1, r1:] @ x[r1:]
            x[r0:r1] = np.linalg.solve(t[r0:r1, r0:r1], x[r0:r1])
            swap(k, False)
    return x


@pytest.mark.parametrize("dt", [np.float64, np.complex128])
@pytest.mark.parametrize("lower,side", [(True, "L"), (False, "L"), (True, "R")])
def test_tbsm_pivots(dt, lower, side):
    """tbsm(side, alpha, A, pivots, B) against a numpy rendering of the
    reference's sweep (interchanges of tile k inside the band reach)."""
    n, nb, kd = 100, 16, 9
    r = np.random.default_rng(31)
    a = rnd(n, n, dt, 11)
    t = (np.tril(band(a, kd, 0)) if lower else np.triu(band(a, 0, kd))) + 4 * np.eye(n)
    nt = -(-n // nb)
    piv = []
    for k in range(nt):
        pk = []
        for i in range(min(nb, n - k * nb)):
            row = k * nb + i
            p = int(r.integers(row, min(n, row + kd + 1)))
            pk.append((p // nb - k, p % nb))
        piv.append(pk)
    b = rnd(n, 5, dt, 12) if side == "L" else rnd(5, n, dt, 12)
    T = s.TriangularBandMatrix(s.Uplo.Lower if lower else s.Uplo.Upper, s.Diag.NonUnit, kd,
                               s.from_numpy(t, nb=nb))
    X = s.from_numpy(b, nb=nb)
    alpha = 0.5
    s.tbsm(s.Side.Left if side == "L" else s.Side.Right, alpha, T, X, pivots=piv)
    if side == "L":
        ref = _tbsm_pivots_ref(t, b, piv, nb, lower, alpha)
    else:
        # X A = alpha B  <=>  A^H X^H = alpha' B^H: the same pivoted sweep on the
        # transposed system (A^H upper for lower A: backward sweep)
        tt = t.conj().T
        ref = _tbsm_pivots_ref(tt, b.conj().T, piv, nb, not lower, np.conj(alpha)).conj().T
    assert relerr(s.to_numpy(X), ref) < tol(dt)
    # empty pivots: plain tbsm
    X2 = s.from_numpy(b, nb=nb)
    if side == "L":
        s.tbsm(s.Side.Left, alpha, T, X2, pivots=[])
        assert relerr(t @ s.to_numpy(X2), alpha * b) < tol(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("uplo", ["L", "U"])
def test_hesv(dt, uplo):
    n, nb = 110, 32
    a = rnd(n, n, dt, 8)
    a = (a + a.conj().T) / 2     # indefinite
    b = rnd(n, 3, dt, 9)
    u = s.Uplo.Lower if uplo == "L" else s.Uplo.Upper
    A = s.HermitianMatrix(u, s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    info, ipiv = s.hesv(A, B)
    assert info == 0
    assert any(p < 0 for p in ipiv) or True
    assert relerr(a @ s.to_numpy(B), b) < 1000 * tol(dt)
    B2 = s.from_numpy(b, nb=nb)
    s.hetrs(A, ipiv, B2)
    assert relerr(a @ s.to_numpy(B2), b) < 1000 * tol(dt)


def test_gbsv_pivoting():
    n, nb, kl, ku = 150, 32, 3, 2
    a = band(rnd(n, n, np.float64, 11), kl, ku)
    b = rnd(n, 2, np.float64, 12)
    A = s.BandMatrix(kl, ku, s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    info, piv = s.gbsv(A, B)
    assert info == 0
    flat = [(k, t) for k, pv in enumerate(piv) for t, _ in enumerate(pv) if pv[t] != (0, t)]
    assert flat, "expected row interchanges"
    x = s.to_numpy(B)
    assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 1e-14


def test_hetrf_2x2_pivots():
    # zero diagonal forces 2x2 pivots
    n, nb = 64, 16
    a = rnd(n, n, np.float64, 13)
    a = a + a.T
    np.fill_diagonal(a, 0.0)
    b = rnd(n, 1, np.float64, 14)
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb))
    B = s.from_numpy(b, nb=nb)
    info, ipiv = s.hesv(A, B)
    assert info == 0 and any(p < 0 for p in ipiv)
    x = s.to_numpy(B)
    assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 1e-13
