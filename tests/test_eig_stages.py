"""Stage-level two-stage eigen/SVD API (reference slate.hh:1050-1334 and
test/test_hb2st.cc, test_tb2bd.cc, test_stedc*.cc, test_steqr2.cc,
test_bdsqr.cc, test_unmtr_hb2st.cc): each stage is chained by hand and the
result checked against numpy (fp64/complex128 oracles), plus the real
symmetric aliases and the gels variants."""
import numpy as np
import pytest

import slate_d35_amd as s
from helpers import rnd, relerr


def herm(n, dt, seed):
    a = rnd(n, n, dt, seed)
    return (a + a.conj().T) / 2


@pytest.mark.parametrize("dt", [np.float64, np.complex128])
@pytest.mark.parametrize("solver", ["stedc", "steqr2"])
def test_heev_by_stages(dt, solver):
    n, nb = 96, 16
    a = herm(n, dt, 1)
    F = s.from_numpy(a, nb=nb)
    Ts = s.he2hb(F)                                   # band of width nb in F
    band = np.tril(s.to_numpy(F))
    band = np.where(np.subtract.outer(np.arange(n), np.arange(n)) <= nb, band, 0)
    Hb = s.HermitianBandMatrix(s.Uplo.Lower, nb, s.from_numpy(band, nb=nb))
    d, e, V = s.hb2st_band(Hb)
    ref = np.linalg.eigvalsh(a)
    Zr = s.from_numpy(np.eye(n), nb=nb)               # real tridiagonal eigenvectors
    if solver == "stedc":
        lam = s.stedc_matrix(d, e, Zr)
    else:
        lam = s.steqr2(s.Job.Vec, d, e, Zr)
    assert np.abs(np.sort(lam) - ref).max() < 1e-12 * np.abs(ref).max()
    Z = s.from_numpy(s.to_numpy(Zr).astype(dt), nb=nb)
    s.unmtr_hb2st(s.Side.Left, s.Op.NoTrans, V, Z)   # Z := Q2 Z
    s.unmtr_he2hb(s.Side.Left, s.Op.NoTrans, F, Ts, Z)  # Z := Q1 Z
    z = s.to_numpy(Z)
    assert relerr(a @ z, z * lam[None, :]) < 1e-12
    assert np.abs(z.conj().T @ z - np.eye(n)).max() < 1e-12


def test_sterf_and_stedc_stages():
    n = 80
    rng = np.random.default_rng(3)
    d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
    t = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    ref = np.linalg.eigvalsh(t)
    assert np.abs(np.sort(s.sterf(d, e)) - ref).max() < 1e-12
    Q = s.from_numpy(np.zeros((n, n)), nb=32)
    lam = s.stedc_matrix(d, e, Q)
    q = s.to_numpy(Q)
    assert np.abs(lam - ref).max() < 1e-12
    assert relerr(t @ q, q * lam[None, :]) < 1e-12


@pytest.mark.parametrize("dt", [np.float64, np.complex128])
def test_svd_by_stages(dt):
    m, n, nb = 70, 48, 16
    a = rnd(m, n, dt, 5)
    W = s.from_numpy(a, nb=nb)
    TU, TV = s.ge2tb(W)
    w = s.to_numpy(W)
    ii, jj = np.meshgrid(np.arange(m), np.arange(n), indexing="ij")
    band = np.where((jj >= ii) & (jj - ii <= nb), w, 0)[:n, :]
    B = s.TriangularBandMatrix(s.Uplo.Upper, s.Diag.NonUnit, nb, s.from_numpy(band, nb=nb))
    d, e, U2, V2 = s.tb2bd_band(B)
    Ub = s.from_numpy(np.eye(n, dtype=dt), nb=nb)
    VTb = s.from_numpy(np.eye(n, dtype=dt), nb=nb)
    sig = s.bdsqr_matrix(s.Job.Vec, s.Job.Vec, d, e, Ub, VTb)
    ref = np.linalg.svd(a, compute_uv=False)
    assert np.abs(np.sort(sig)[::-1] - ref).max() < 1e-12 * ref.max()
    # U = U1 * U2 * Ub ; VT = VTb * V2^H * V1^H
    s.unmbr_tb2bd(s.Side.Left, s.Op.NoTrans, U2, Ub)
    s.unmbr_tb2bd(s.Side.Right, s.Op.ConjTrans, V2, VTb)
    U = s.from_numpy(np.vstack([s.to_numpy(Ub), np.zeros((m - n, n), dt)]), nb=nb)
    s.unmbr_ge2tb(s.Side.Left, s.Op.NoTrans, W, TU, U)
    s.unmbr_ge2tb(s.Side.Right, s.Op.NoTrans, W, TV, VTb)
    u, vt = s.to_numpy(U), s.to_numpy(VTb)
    assert relerr((u * sig[None, :]) @ vt, a) < 1e-12


def test_real_symmetric_aliases():
    n, nb = 64, 16
    a = herm(n, np.float64, 7)
    Z = s.from_numpy(np.zeros((n, n)), nb=nb)
    lam = s.syev(s.SymmetricMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb)), Z)
    assert np.abs(lam - np.linalg.eigvalsh(a)).max() < 1e-12
    b = herm(n, np.float64, 8) + n * np.eye(n)
    lam2 = s.sygv(1, s.SymmetricMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb)),
                  s.SymmetricMatrix(s.Uplo.Lower, s.from_numpy(b, nb=nb)))
    import scipy.linalg as sl
    assert np.abs(lam2 - sl.eigh(a, b, eigvals_only=True)).max() < 1e-10
    rhs = rnd(n, 3, np.float64, 9)
    B = s.from_numpy(rhs, nb=nb)
    info, ipiv = s.sysv(s.SymmetricMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb)), B)
    assert info == 0 and relerr(a @ s.to_numpy(B), rhs) < 1e-10


@pytest.mark.parametrize("variant", ["qr", "cholqr"])
def test_gels_variants(variant):
    m, n, nrhs, nb = 120, 40, 3, 16
    a = rnd(m, n, np.float64, 11)
    b = rnd(m, nrhs, np.float64, 12)
    A = s.from_numpy(a, nb=nb)
    BX = s.from_numpy(b, nb=nb)
    if variant == "qr":
        s.gels_qr(A, BX)
    else:
        R = s.from_numpy(np.zeros((n, n)), nb=nb)
        s.gels_cholqr(A, R, BX)
    x = s.to_numpy(BX)[:n]
    ref = np.linalg.lstsq(a, b, rcond=None)[0]
    assert relerr(x, ref) < 1e-10


def test_gesvd_alias():
    a = rnd(50, 30, np.float64, 13)
    sig = s.gesvd(s.from_numpy(a, nb=16))
    assert np.abs(sig - np.linalg.svd(a, compute_uv=False)).max() < 1e-12
