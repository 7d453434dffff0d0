"""Multi-device matrices: one process, its matrix spread over the devices of an
in-process group (reference: one MPI rank gives its tiles to all of its GPUs,
tileDevice = func::device_1d_grid, include/slate/internal/MatrixStorage.hh:
503-506; Matrix::fromDevices(Aarray, num_devices), include/slate/Matrix.hh:
396-404 and 529-563).

Drivers called with such matrices run on the group's ranks directly on each
rank's part: a factor-then-solve sequence moves no matrix data between the
caller and the ranks (inproc_copy_bytes stays put) -- unlike the copy-in /
copy-out path for one-GPU matrices.  These tests run in host mode here (no
GPU: the parts are host arrays); test_gpu.py repeats the core ones on the
device.
"""
import numpy as np
import pytest

import slate_d35_amd as s
from slate_d35_amd import _slate

NR = 4


def rnd(m, n, seed, dtype=np.float64):
    r = np.random.default_rng(seed)
    a = r.standard_normal((m, n))
    if np.dtype(dtype).kind == "c":
        a = a + 1j * r.standard_normal((m, n))
    return a.astype(dtype)


def counters():
    return _slate.inproc_copy_bytes(), _slate.inproc_run_count()


def test_multi_device_layout_and_gather():
    a = rnd(200, 150, 1)
    A = s.to_multi_device(a, nb=32, num_devices=NR)
    assert A.is_multi_device and A.num_parts == NR
    assert np.array_equal(s.to_numpy(A), a)
    out = np.zeros((200, 150), order="F")
    A.gather_into(out)
    assert np.array_equal(out, a)
    assert s.norm(s.Norm.Fro, A) == pytest.approx(np.linalg.norm(a))
    # views: a sub-matrix and a transpose see the same data
    assert s.norm(s.Norm.One, A.sub(1, 3, 0, 2)) == pytest.approx(np.abs(a[32:128, 0:96]).sum(0).max())
    assert s.norm(s.Norm.Inf, s.transpose(A)) == pytest.approx(np.abs(a.T).sum(1).max())


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_lu_factor_then_solve_twice_no_copies(dtype):
    n, nb = 260, 32
    a = rnd(n, n, 2, dtype) + n * np.eye(n)
    b1, b2 = rnd(n, 3, 3, dtype), rnd(n, 5, 4, dtype)
    A = s.to_multi_device(a, nb=nb, num_devices=NR)
    B1 = s.to_multi_device(b1, nb=nb, num_devices=NR)
    B2 = s.to_multi_device(b2, nb=nb, num_devices=NR)
    c0, r0 = counters()
    info, piv = s.getrf(A)
    assert info == 0
    s.getrs(A, piv, B1)
    s.getrs(A, piv, B2)
    c1, r1 = counters()
    assert c1 == c0, "a driver on multi-device matrices copied data"
    assert r1 - r0 == 3                      # one in-process run per driver
    for b, B in ((b1, B1), (b2, B2)):
        x = s.to_numpy(B)
        assert np.abs(a @ x - b).max() / (np.abs(a).max() * np.abs(x).max() * n) < 1e-14


def test_cholesky_and_trsm_herk_gemm():
    n, nb = 230, 32
    g = rnd(n, n, 5)
    a = g @ g.T + n * np.eye(n)
    b = rnd(n, 4, 6)
    A = s.HermitianMatrix(s.Uplo.Lower, s.to_multi_device(a, nb=nb, num_devices=NR))
    B = s.to_multi_device(b, nb=nb, num_devices=NR)
    c0, _ = counters()
    assert s.potrf(A) == 0
    s.potrs(A, B)
    assert counters()[0] == c0
    x = s.to_numpy(B)
    assert np.abs(a @ x - b).max() < 1e-9
    # trsm with the factor: L^{-1} b
    L = np.tril(s.to_numpy(s.general(A)))
    B2 = s.to_multi_device(b, nb=nb, num_devices=NR)
    s.trsm(s.Side.Left, 1.0, s.TriangularMatrix(s.Uplo.Lower, s.Diag.NonUnit, s.general(A)), B2)
    assert np.allclose(s.to_numpy(B2), np.linalg.solve(L, b))
    # herk C = G^T G (lower) and gemm C = G G
    G = s.to_multi_device(g, nb=nb, num_devices=NR)
    C = s.HermitianMatrix(s.Uplo.Lower, s.to_multi_device(np.zeros((n, n)), nb=nb, num_devices=NR))
    s.herk(1.0, s.conj_transpose(G), 0.0, C)
    assert np.allclose(np.tril(s.to_numpy(s.general(C))), np.tril(g.T @ g))
    D = s.to_multi_device(np.zeros((n, n)), nb=nb, num_devices=NR)
    s.gemm(1.0, G, G, 0.0, D)
    assert np.allclose(s.to_numpy(D), g @ g)


def test_qr_least_squares_and_unmqr():
    m, n, nb = 300, 120, 32
    a = rnd(m, n, 7)
    b = rnd(m, 2, 8)
    A = s.to_multi_device(a, nb=nb, num_devices=NR)
    BX = s.to_multi_device(b, nb=nb, num_devices=NR)
    c0, _ = counters()
    T = s.gels(A, BX)
    assert counters()[0] == c0
    x = s.to_numpy(BX)[:n]
    assert np.allclose(x, np.linalg.lstsq(a, b, rcond=None)[0])
    assert all(t.is_multi_device for t in T)
    # Q^H Q = I through the distributed T factors
    A2 = s.to_multi_device(a, nb=nb, num_devices=NR)
    T2 = s.geqrf(A2)
    C = s.to_multi_device(np.eye(m)[:, :n].copy(), nb=nb, num_devices=NR)
    s.unmqr(s.Side.Left, s.Op.NoTrans, A2, T2, C)      # C = Q(:, :n)
    q = s.to_numpy(C)
    assert np.allclose(q.T @ q, np.eye(n), atol=1e-12)
    r = np.triu(s.to_numpy(A2)[:n])
    assert np.allclose(q @ r, a)


def test_mixed_precision_and_eig_svd():
    n, nb = 200, 32
    a = rnd(n, n, 9) + 4 * np.sqrt(n) * np.eye(n)
    b = rnd(n, 2, 10)
    A = s.to_multi_device(a, nb=nb, num_devices=NR)
    B = s.to_multi_device(b, nb=nb, num_devices=NR)
    X = s.to_multi_device(np.zeros((n, 2)), nb=nb, num_devices=NR)
    c0, _ = counters()
    info, piv, it = s.gesv_mixed(A, B, X)
    assert info == 0 and counters()[0] == c0
    assert np.abs(a @ s.to_numpy(X) - b).max() < 1e-9
    h = a + a.T
    H = s.HermitianMatrix(s.Uplo.Lower, s.to_multi_device(h, nb=nb, num_devices=NR))
    Z = s.to_multi_device(np.zeros((n, n)), nb=nb, num_devices=NR)
    w = s.heev(H, Z)
    assert np.allclose(w, np.linalg.eigvalsh(h))
    z = s.to_numpy(Z)
    assert np.allclose(h @ z, z * w, atol=1e-9)
    S = s.svd(s.to_multi_device(a, nb=nb, num_devices=NR))
    assert np.allclose(S, np.linalg.svd(a, compute_uv=False))


def test_from_devices_reference_layout():
    """fromDevices(Aarray, num_devices): tile column j on device j % nd, each
    array holding its devices' tile columns side by side (host arrays here)."""
    m, n, nb, nd = 100, 90, 16, 3
    a = rnd(m, n, 11)
    nt = -(-n // nb)
    cols = [[j for j in range(nt) if j % nd == d] for d in range(nd)]
    arrays = []
    for d in range(nd):
        idx = np.concatenate([np.arange(j * nb, min(n, (j + 1) * nb)) for j in cols[d]]) if cols[d] else []
        arrays.append(np.asfortranarray(a[:, idx]) if len(idx) else np.zeros((m, 1), order="F"))
    A = s.from_devices(m, n, [x.ctypes.data for x in arrays], m, nb)
    assert A.is_multi_device and A.num_parts == nd
    assert np.array_equal(s.to_numpy(A), a)
    s.scale(2.0, 1.0, A)                      # in place on the caller's arrays
    assert np.array_equal(arrays[1], 2 * np.asfortranarray(a[:, np.concatenate(
        [np.arange(j * nb, min(n, (j + 1) * nb)) for j in cols[1]])]))


def test_unsupported_driver_fails_loudly():
    A = s.to_multi_device(rnd(64, 64, 12), nb=16, num_devices=NR)
    with pytest.raises(Exception, match="multi-device"):
        A.get_local()
