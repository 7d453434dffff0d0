"""GPU tests: gfx950 kernels vs fp64 torch/numpy references and device-target
drivers (reference unit_test/test_Tile_kernels.cc, test_internal_blas.cc and
the tester's residual checks)."""
import os

import numpy as np
import pytest

import slate_d35_amd as s
from helpers import DTYPES, rnd, tol, relerr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torch():
    import torch
    return torch


def _native_loaded():
    import slate_d35_amd._slate as m
    assert m.__file__.endswith(".so")
    assert s.device_available(), "native HIP path must be active on a GPU box"


def test_native_extension_loaded():
    _native_loaded()


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("N", "T"), ("T", "N"), ("T", "T"), ("C", "N")])
def test_gemm_kernel(dtype, ta, tb):
    torch = _torch()
    m, n, k = 300, 257, 129
    if ta == "C" and not np.iscomplexobj(np.zeros(1, dtype)):
        ta = "T"
    a = rnd(m, k, dtype, 1) if ta == "N" else rnd(k, m, dtype, 1)
    b = rnd(k, n, dtype, 2) if tb == "N" else rnd(n, k, dtype, 2)
    c = rnd(m, n, dtype, 3)
    # column-major matrices = row-major tensors of the transposes
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    alpha, beta = dtype(0.5), dtype(-2.0)
    s.ops.gemm(ta, tb, alpha, tA, tB, beta, tC)
    opa = a if ta == "N" else (a.T if ta == "T" else a.conj().T)
    opb = b if tb == "N" else b.T
    ref = alpha * opa.astype(np.complex128 if np.iscomplexobj(a) else np.float64) @ opb + beta * c
    assert relerr(tC.cpu().numpy().T, ref) < tol(dtype)


@pytest.mark.parametrize("n", [40, 300])
def test_gemm_herk_k0_scales_by_beta(n):
    """k == 0: C = beta C (BLAS semantics) for gemm and herk on the device."""
    torch = _torch()
    m = 257
    c = rnd(m, n, np.float64, 30)
    tA = torch.zeros((0, m), dtype=torch.float64).cuda()
    tB = torch.zeros((n, 0), dtype=torch.float64).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.gemm("N", "N", 1.0, tA, tB, -0.5, tC)
    assert relerr(tC.cpu().numpy().T, -0.5 * c) < 1e-15
    h = rnd(n, n, np.float64, 31)
    tH = torch.from_numpy(np.ascontiguousarray(h.T)).cuda()
    tK = torch.zeros((0, n), dtype=torch.float64).cuda()
    s.ops.herk("L", "N", 1.0, tK, 3.0, tH)
    got = tH.cpu().numpy().T
    low = np.tril(np.ones((n, n), bool))
    assert relerr(got[low], 3.0 * h[low]) < 1e-15
    np.testing.assert_array_equal(got[~low], h[~low])


def test_gemm_nn_long_k_packed_a():
    """Long-K NN products (K > 2048, m, n >= 4096) run as TN on a transposed
    copy of A (local_blas.cc dgemm); against numpy."""
    torch = _torch()
    m, n, k = 4200, 4100, 2300
    a, b, c = rnd(m, k, np.float64, 24), rnd(k, n, np.float64, 25), rnd(m, n, np.float64, 26)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.gemm("N", "N", 0.75, tA, tB, 2.0, tC)
    assert relerr(tC.cpu().numpy().T, 0.75 * a @ b + 2.0 * c) < 1e-13


def test_gemm_nn_long_k_packed_a_sliced(monkeypatch):
    """The transposed copy of A is made in K slices bounded by
    SLATE_GEMM_PACK_BYTES (later slices accumulate with beta = 1)."""
    torch = _torch()
    m, n, k = 4200, 4100, 6000
    monkeypatch.setenv("SLATE_GEMM_PACK_BYTES", str(4200 * 2304 * 8))   # 2304-row slices
    a, b, c = rnd(m, k, np.float64, 27), rnd(k, n, np.float64, 28), rnd(m, n, np.float64, 29)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.gemm("N", "N", -1.25, tA, tB, 0.5, tC)
    assert relerr(tC.cpu().numpy().T, -1.25 * a @ b + 0.5 * c) < 1e-13


@pytest.mark.parametrize("k", [256, 512, 2048])
def test_gemm_nn_rank_nb_packed(k):
    """Rank-nb NN products (m >= 4096, n >= 1024, 256 <= K <= 2048) run as NT
    products on a transposed copy of B (local_blas.cc dgemm); against numpy."""
    torch = _torch()
    m, n = 4160, 1100
    a, b, c = rnd(m, k, np.float64, 21), rnd(k, n, np.float64, 22), rnd(m, n, np.float64, 23)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.gemm("N", "N", 1.5, tA, tB, -0.5, tC)
    assert relerr(tC.cpu().numpy().T, 1.5 * a @ b - 0.5 * c) < 1e-13


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("uplo", ["L", "U"])
@pytest.mark.parametrize("n,k,op", [(333, 97, "N"), (300, 5000, "N"), (300, 5000, "C")])   # k = 5000: split-K triangular path
def test_herk_kernel(dtype, uplo, n, k, op):
    torch = _torch()
    a = rnd(n, k, dtype, 4) if op == "N" else rnd(k, n, dtype, 4)
    c = rnd(n, n, dtype, 5)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.herk(uplo, op, -1.0, tA, 1.0, tC)
    got = tC.cpu().numpy().T
    a64 = a.astype(np.float64)
    ref = c - (a64 @ a64.T if op == "N" else a64.T @ a64)
    mask = np.tril(np.ones((n, n), bool)) if uplo == "L" else np.triu(np.ones((n, n), bool))
    assert relerr(got[mask], ref[mask]) < tol(dtype)
    np.testing.assert_array_equal(got[~mask], c[~mask])  # other triangle untouched


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
@pytest.mark.parametrize("side,uplo,op,diag", [("L", "L", "N", "U"), ("L", "U", "N", "N"), ("R", "L", "C", "N"),
                                               ("R", "U", "N", "N"), ("L", "L", "C", "N")])
def test_trsm_kernel(dtype, side, uplo, op, diag):
    torch = _torch()
    m, n = 700, 300
    na = m if side == "L" else n
    # well-conditioned triangle (random unit triangles are exponentially ill-conditioned)
    t = rnd(na, na, dtype, 6) / na + 2 * np.eye(na, dtype=dtype)
    t = np.tril(t) if uplo == "L" else np.triu(t)
    te = t.copy()
    if diag == "U":
        np.fill_diagonal(te, 1)
    b = rnd(m, n, dtype, 7)
    tT = torch.from_numpy(np.ascontiguousarray(t.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    s.ops.trsm(side, uplo, op, diag, dtype(1), tT, tB)
    x = tB.cpu().numpy().T
    ope = te if op == "N" else te.conj().T
    lhs = ope @ x if side == "L" else x @ ope
    assert relerr(lhs, b) < 1e-10


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
@pytest.mark.parametrize("ta", ["N", "T", "C"])
@pytest.mark.parametrize("nr", [1, 3, 16])
@pytest.mark.parametrize("mk", [(5000, 4099), (37, 20000)])
def test_gemv_kernel(dtype, ta, nr, mk):
    """Few-column gemm (n <= 16) takes the gemv kernels: row-per-lane NoTrans
    and wave-per-row (conj-)transposed, K-chunked for short outputs."""
    torch = _torch()
    if ta == "C" and not np.iscomplexobj(np.zeros(1, dtype)):
        ta = "T"
    m, k = mk
    a = rnd(m, k, dtype, 11) if ta == "N" else rnd(k, m, dtype, 11)
    b = rnd(k, nr, dtype, 12)
    c = rnd(m, nr, dtype, 13)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    alpha, beta = dtype(-1.0), dtype(0.75)
    s.ops.gemm(ta, "N", alpha, tA, tB, beta, tC)
    opa = a if ta == "N" else (a.T if ta == "T" else a.conj().T)
    wide = np.complex128 if np.iscomplexobj(a) else np.float64
    ref = alpha * opa.astype(wide) @ b.astype(wide) + beta * c
    assert relerr(tC.cpu().numpy().T, ref) < tol(dtype)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("uplo,op,diag", [("L", "N", "U"), ("U", "N", "N"), ("L", "T", "U"), ("U", "T", "N")])
@pytest.mark.parametrize("m", [2500, 17000])
def test_trsm_skinny_kernel(dtype, uplo, op, diag, m):
    """Left trsm with few right-hand sides: batched inverse of the BS x BS
    diagonal blocks (BS = 512 / 1024, remainder block separately) + gemv sweep."""
    torch = _torch()
    nr = 2
    t = (rnd(m, m, dtype, 14) / np.sqrt(m) * 0.5 + 2 * np.eye(m)).astype(dtype)
    t = np.tril(t) if uplo == "L" else np.triu(t)
    te = t.astype(np.float64)
    if diag == "U":
        np.fill_diagonal(te, 1)
    b = rnd(m, nr, dtype, 15)
    tT = torch.from_numpy(np.ascontiguousarray(t.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    s.ops.trsm("L", uplo, op, diag, dtype(1), tT, tB)
    x = tB.cpu().numpy().T.astype(np.float64)
    ope = te if op == "N" else te.T
    assert relerr(ope @ x, b) < (1e-12 if dtype == np.float64 else 2e-5)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("uplo,diag", [("L", "U"), ("L", "N"), ("U", "N"), ("U", "U")])
@pytest.mark.parametrize("m,nr", [(17, 5), (32, 300), (64, 129)])
def test_trsm_small_kernel(dtype, uplo, diag, m, nr):
    """Left NoTrans trsm with a small triangle (m <= 64): one-launch
    substitution kernel (lane per right-hand-side column) against numpy."""
    torch = _torch()
    t = (rnd(m, m, dtype, 16) * 0.3 + 2 * np.eye(m)).astype(dtype)
    t = np.tril(t) if uplo == "L" else np.triu(t)
    te = t.astype(np.float64)
    if diag == "U":
        np.fill_diagonal(te, 1)
    b = rnd(m, nr, dtype, 17)
    tT = torch.from_numpy(np.ascontiguousarray(t.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    s.ops.trsm("L", uplo, "N", diag, dtype(1), tT, tB)
    x = tB.cpu().numpy().T.astype(np.float64)
    assert relerr(te @ x, b) < (1e-13 if dtype == np.float64 else 1e-5)


@pytest.mark.parametrize("n", [64, 200, 512, 1000, 2500])
@pytest.mark.parametrize("uplo", ["L", "U"])
def test_potrf_kernel(n, uplo):
    torch = _torch()
    a = s.utils.spd_matrix(n)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info = s.ops.potrf(uplo, tA)
    f = tA.cpu().numpy().T
    if uplo == "L":
        L = np.tril(f)
        assert info == 0 and relerr(L @ L.T, a) < 1e-13
    else:
        U = np.triu(f)
        assert info == 0 and relerr(U.T @ U, a) < 1e-13


@pytest.mark.parametrize("n,bad", [(200, 150), (2500, 2100)])
def test_potrf_kernel_not_spd(n, bad):
    # n = 2500: the failure sits in a recursive split's second half
    torch = _torch()
    a = s.utils.spd_matrix(n)
    a[bad, bad] = -1e6
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info = s.ops.potrf("L", tA)
    assert info == bad + 1


@pytest.mark.parametrize("dt", [np.float64, np.float32, np.complex64, np.complex128])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 130, 700, 1024])
def test_potrf_leaf_all_types(n, dt):
    """Blocked lower potrf: 64-column leaves (factor + A21 solve in one launch
    for sizeof(T) <= 8, the inverse-based leaf for complex128), partial last
    leaves, and the small-tile triangular updates between them."""
    torch = _torch()
    a = s.utils.spd_matrix(n, dtype=dt)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info = s.ops.potrf("L", tA)
    L = np.tril(tA.cpu().numpy().T).astype(np.complex128)
    tol = 1e-5 if dt in (np.float32, np.complex64) else 1e-13
    assert info == 0 and relerr(L @ L.conj().T, a) < tol
    if n >= 130:
        for bad in (0, 63, 64, 100, n - 1):
            b = a.copy()
            b[bad, bad] = -1e6
            tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
            assert s.ops.potrf("L", tB) == bad + 1, bad


@pytest.mark.parametrize("dt", [np.float64, np.float32, np.complex64, np.complex128])
@pytest.mark.parametrize("n", [1, 31, 64, 100, 512, 700])
def test_lu_sign_device(n, dt):
    """Sign-modified LU without pivoting (Householder reconstruction step):
    L U = A + diag(s) with |s_k| = 1 and |U_kk| >= 1 for A = -Q11 of an
    orthonormal Q."""
    torch = _torch()
    q, _ = np.linalg.qr(rnd(2 * n, n, dt, 21))
    a = -q[:n, :n]
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    sg = np.array(s.ops.lu_sign(tA))
    f = tA.cpu().numpy().T.astype(np.complex128)
    L = np.tril(f, -1) + np.eye(n)
    U = np.triu(f)
    tol = 1e-5 if dt in (np.float32, np.complex64) else 1e-13
    assert np.allclose(np.abs(sg), 1.0)
    assert np.abs(np.diag(U)).min() >= 1.0 - tol
    assert np.abs(L @ U - (a + np.diag(sg))).max() < tol * max(1, n) ** 0.5


@pytest.mark.parametrize("m,n", [(1000, 64), (4096, 256), (777, 100), (512, 512)])
def test_getrf_panel_kernel(m, n):
    torch = _torch()
    a = rnd(m, n, np.float64, 8)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info, ipiv = s.ops.getrf_panel(tA)
    f = tA.cpu().numpy().T
    k = min(m, n)
    L = np.tril(f[:, :k], -1) + np.eye(m, k)
    U = np.triu(f[:k, :])
    pa = a.copy()
    for j, p in enumerate(ipiv):
        pa[[j, p]] = pa[[p, j]]
    assert info == 0
    assert relerr(L @ U, pa) < 1e-13
    # partial pivoting: |L| <= 1
    assert np.abs(L).max() <= 1.0 + 1e-12
    # pivots match a reference partial-pivoting LU (first column at least)
    assert ipiv[0] == int(np.argmax(np.abs(a[:, 0])))


@pytest.mark.parametrize("dt", [np.float64, np.complex128, np.float32])
@pytest.mark.parametrize("m,n", [(1000, 64), (8192, 256), (3000, 100), (70000, 32), (300, 300)])
def test_getrf_panel_tournament(m, n, dt):
    """CALU panel: P A = L U with the pivots chosen by the device tournament;
    |L| stays modest (tournament growth) and the factorization is exact."""
    torch = _torch()
    a = rnd(m, n, dt, 18)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info, ipiv = s.ops.getrf_panel(tA, tournament=True)
    f = tA.cpu().numpy().T
    k = min(m, n)
    L = np.tril(f[:, :k], -1) + np.eye(m, k)
    U = np.triu(f[:k, :])
    pa = a.copy()
    for j, p in enumerate(ipiv):
        pa[[j, p]] = pa[[p, j]]
    assert info == 0
    tol = 1e-4 if dt == np.float32 else 1e-12
    assert relerr(L @ U, pa) < tol
    assert np.abs(L).max() < 8.0
    # first pivot is still the column's absolute maximum (the tournament's
    # first round at every node is a plain max search)
    assert ipiv[0] == int(np.argmax(np.abs(a[:, 0].real) + np.abs(a[:, 0].imag)))


def test_getrf_panel_tournament_singular():
    torch = _torch()
    a = rnd(2000, 64, np.float64, 19)
    a[:, 5] = 0.0
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    info, _ = s.ops.getrf_panel(tA, tournament=True)
    assert info == 6


@pytest.mark.parametrize("m,n", [(1000, 64), (2048, 256), (500, 100), (8, 64), (20, 100), (64, 130), (33, 40)])
def test_geqrf_panel_kernel(m, n):
    torch = _torch()
    a = rnd(m, n, np.float64, 9)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tau, Tm = s.ops.geqrf_panel(tA)
    f = tA.cpu().numpy().T
    k = min(m, n)
    V = np.tril(f[:, :k], -1) + np.eye(m, k)
    R = np.triu(f[:k, :])
    T = np.array(Tm).reshape(k, k, order="F")
    Q = np.eye(m) - V @ T @ V.T
    assert relerr(Q[:, :k] @ R, a) < 1e-13
    assert np.abs(Q.T @ Q - np.eye(m)).max() < 1e-12


# ---------------------------------------------------------------- drivers
@pytest.mark.parametrize("dtype", DTYPES)
def test_gemm_driver_device(dtype):
    m, n, k, nb = 400, 300, 200, 128
    a, b, c = rnd(m, k, dtype, 1), rnd(k, n, dtype, 2), rnd(m, n, dtype, 3)
    A, B, C = (s.from_numpy(x, nb=nb, target="d") for x in (a, b, c))
    s.gemm(dtype(1.5), A, B, dtype(0.5), C, target="d")
    assert relerr(s.to_numpy(C), 1.5 * a @ b + 0.5 * c) < tol(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("uplo", [s.Uplo.Lower, s.Uplo.Upper])
def test_potrf_driver_device(dtype, uplo):
    n, nb = 700, 128
    a = s.utils.spd_matrix(n, dtype=dtype)
    A = s.from_numpy(a, nb=nb, target="d")
    info = s.potrf(s.HermitianMatrix(uplo, A), target="d", lookahead=2)
    f = s.to_numpy(A)
    if uplo == s.Uplo.Lower:
        L = np.tril(f); rec = L @ L.conj().T
    else:
        U = np.triu(f); rec = U.conj().T @ U
    assert info == 0 and relerr(rec, a) < 10 * tol(dtype)


@pytest.mark.parametrize("side", [s.Side.Left, s.Side.Right])
def test_trsm_driver_device(side):
    m, n, nb = 600, 500, 128
    na = m if side == s.Side.Left else n
    t = np.tril(rnd(na, na, np.float64, 5)) + na * np.eye(na)
    b = rnd(m, n, np.float64, 6)
    T = s.TriangularMatrix(s.Uplo.Lower, s.Diag.NonUnit, s.from_numpy(t, nb=nb, target="d"))
    B = s.from_numpy(b, nb=nb, target="d")
    s.trsm(side, 1.0, T, B, target="d")
    x = s.to_numpy(B)
    assert relerr(t @ x if side == s.Side.Left else x @ t, b) < 1e-12


def test_norm_device():
    a = rnd(500, 300, np.float64, 11)
    A = s.from_numpy(a, nb=128, target="d")
    for kind, npk in [(s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro")]:
        assert abs(s.norm(kind, A, target="d") - np.linalg.norm(a, npk)) < 1e-10 * np.linalg.norm(a, npk)
    assert s.norm(s.Norm.Max, A, target="d") == np.abs(a).max()


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32])
def test_norm_device_wide_block(dtype):
    # local block wider than one column chunk: 2-D row-sum kernel + in-order chunk reduction
    a = rnd(333, 1700, dtype, 12)
    A = s.from_numpy(a, nb=96, target="d")
    rt = 1e-5 if dtype == np.float32 else 1e-12
    for kind, npk in [(s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro")]:
        ref = np.linalg.norm(a.astype(np.complex128 if np.iscomplexobj(a) else np.float64), npk)
        assert abs(s.norm(kind, A, target="d") - ref) < rt * ref, kind
    assert abs(s.norm(s.Norm.Max, A, target="d") - np.abs(a).max()) <= rt * np.abs(a).max()


def test_generate_matrix_device_matches_host():
    for kind in ("rands", "spd"):
        A = s.Matrix(300, 300, 64); A.insertLocalTiles(s.Target.Devices)
        B = s.Matrix(300, 300, 64); B.insertLocalTiles(s.Target.Host)
        s._slate.generate_matrix_d(kind, A, 5, -1.0, s.opts("d"))
        s._slate.generate_matrix_d(kind, B, 5, -1.0, s.opts("h"))
        np.testing.assert_array_equal(s.to_numpy(A), s.to_numpy(B))


@pytest.mark.parametrize("kind", ["randn", "rand_dominant", "chebspec", "orthog", "kms", "riemann", "gfpp",
                                  "diag_geo", "svd_arith", "heev", "poev_cluster0", "geev"])
@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_matgen_kinds_device_match_host(kind, dtype):
    from slate_d35_amd.utils import matgen as mg
    out = []
    for tg in ("d", "h"):
        A = s.Matrix(260, 260, 64, dtype); A.insertLocalTiles(s.target_of(tg))
        S, _ = mg.generate_matrix(kind, A, seed=3, cond=1e3, target=tg)
        out.append((s.to_numpy(A), S))
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-14)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("mn", [(700, 700), (900, 500), (500, 900), (1500, 1300)])
def test_getrf_driver_device(dtype, mn):
    m, n = mn
    nb = 128
    a = rnd(m, n, dtype, 21)
    A = s.from_numpy(a, nb=nb, target="d")
    info, piv = s.getrf(A, target="d", lookahead=1)
    f = s.to_numpy(A)
    k = min(m, n)
    L = np.tril(f[:, :k], -1) + np.eye(m, k)
    U = np.triu(f[:k, :])
    ip = [kk * nb + ti * nb + off for kk, pv in enumerate(piv) for (ti, off) in pv]
    pa = a.copy()
    for j, p_ in enumerate(ip):
        pa[[j, p_]] = pa[[p_, j]]
    assert info == 0 and relerr(L @ U, pa) < 10 * tol(dtype)


@pytest.mark.parametrize("method", ["ppiv", "tntpiv"])
@pytest.mark.parametrize("nb", [1280, 2048])
def test_getrf_device_wide_tiles(method, nb):
    """Tiles wider than 1024: the per-step row permutation then has more than
    2048 (dst, src) pairs and takes the LDS-staged permute kernel (a second
    register pass used to read rows the first pass had overwritten)."""
    n = 3000
    a = rnd(n, n, np.float64, 27)
    A = s.from_numpy(a, nb=nb, target="d")
    info, piv = s.getrf(A, target="d", method_lu=method)
    f = s.to_numpy(A)
    L = np.tril(f, -1) + np.eye(n)
    U = np.triu(f)
    ip = [kk * nb + ti * nb + off for kk, pv in enumerate(piv) for (ti, off) in pv]
    pa = a.copy()
    for j, p_ in enumerate(ip):
        pa[[j, p_]] = pa[[p_, j]]
    assert info == 0 and relerr(L @ U, pa) < 1e-12


@pytest.mark.parametrize("n,nrhs", [(1000, 4), (5000, 1)])
def test_gesv_mixed_device(n, nrhs):
    nb = 128
    a = rnd(n, n, np.float64, 31)
    b = rnd(n, nrhs, np.float64, 32)
    A, B = s.from_numpy(a, nb=nb, target="d"), s.from_numpy(b, nb=nb, target="d")
    X = s.from_numpy(np.zeros_like(b), nb=nb, target="d")
    info, piv, it = s.gesv_mixed(A, B, X, target="d")
    x = s.to_numpy(X)
    assert info == 0 and it >= 0
    assert np.linalg.norm(a @ x - b, 1) / (np.linalg.norm(a, 1) * np.linalg.norm(x, 1)) < 1e-15 * n


def test_posv_device():
    n, nb = 900, 128
    a = s.utils.spd_matrix(n)
    b = rnd(n, 3, np.float64, 33)
    A, B = s.from_numpy(a, nb=nb, target="d"), s.from_numpy(b, nb=nb, target="d")
    assert s.posv(s.HermitianMatrix(s.Uplo.Lower, A), B, target="d") == 0
    assert relerr(a @ s.to_numpy(B), b) < 1e-12


@pytest.mark.parametrize("mn", [(700, 700), (1000, 400)])
def test_geqrf_driver_device(mn):
    m, n = mn
    nb = 128
    a = rnd(m, n, np.float64, 41)
    A = s.from_numpy(a, nb=nb, target="d")
    T = s.geqrf(A, target="d")
    k = min(m, n)
    R = np.triu(s.to_numpy(A)[:k, :])
    C = s.from_numpy(a, nb=nb, target="d")
    s.unmqr(s.Side.Left, s.Op.ConjTrans, A, T, C, target="d")
    qa = s.to_numpy(C)
    assert relerr(qa[:k], R) < 1e-13
    if m > k:
        assert np.abs(qa[k:]).max() < 1e-12


def test_gels_device():
    m, n = 900, 300
    a, b = rnd(m, n, np.float64, 42), rnd(m, 2, np.float64, 43)
    A, B = s.from_numpy(a, nb=128, target="d"), s.from_numpy(b, nb=128, target="d")
    s.gels(A, B, target="d")
    x = s.to_numpy(B)[:n]
    assert relerr(x, np.linalg.lstsq(a, b, rcond=None)[0]) < 1e-12


@pytest.mark.parametrize("ta", ["N", "T"])
def test_gemm_splitk_kernel(ta):
    """small output, long K -> split-K path"""
    torch = _torch()
    m, n, k = 200, 96, 20000
    a = rnd(m, k, np.float64, 51) if ta == "N" else rnd(k, m, np.float64, 51)
    b = rnd(k, n, np.float64, 52)
    c = rnd(m, n, np.float64, 53)
    tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
    tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
    tC = torch.from_numpy(np.ascontiguousarray(c.T)).cuda()
    s.ops.gemm(ta, "N", 2.0, tA, tB, 0.5, tC)
    opa = a if ta == "N" else a.T
    assert relerr(tC.cpu().numpy().T, 2.0 * opa @ b + 0.5 * c) < 1e-12


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_heev_device(dtype):
    n, nb = 300, 64
    a = rnd(n, n, dtype, 31)
    a = (a + a.conj().T) / 2
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb, target="d"))
    Z = s.from_numpy(np.zeros((n, n), dtype), nb=nb, target="d")
    w = s.heev(A, Z, target="d")
    assert np.allclose(w, np.linalg.eigvalsh(a), atol=1e-10 * n)
    z = s.to_numpy(Z)
    assert np.linalg.norm(a @ z - z * w) / (np.linalg.norm(a) * n) < 1e-12


@pytest.mark.parametrize("n,nb", [(2200, 48), (8192, 256)])
def test_heev_device_stage2_fused(n, nb):
    """Fused stage-2 back-transform (hb2st_apply.hip): several 512-group
    chunks, kd < 64 (nb = 48) and the 32-column slices (n = 8192); residual
    and orthogonality checked on the GPU."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.rand(n, n, dtype=torch.float64, device="cuda", generator=g) * 2 - 1
    a = (a + a.T) / 2
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a.cpu().numpy(), nb=nb, target="d"))
    Z = s.from_numpy(np.zeros((n, n)), nb=nb, target="d")
    w = torch.tensor(np.asarray(s.heev(A, Z, target="d")), device="cuda")
    z = torch.tensor(s.to_numpy(Z), device="cuda")
    an = torch.linalg.norm(a)
    assert float(torch.linalg.norm(a @ z - z * w) / (an * n)) < 1e-13
    assert float(torch.linalg.norm(z.T @ z - torch.eye(n, dtype=torch.float64, device="cuda")) / n) < 1e-13


def test_svd_device():
    m, n, nb = 320, 200, 64
    a = rnd(m, n, np.float64, 32)
    A = s.from_numpy(a, nb=nb, target="d")
    U = s.from_numpy(np.zeros((m, n)), nb=nb, target="d")
    VT = s.from_numpy(np.zeros((n, n)), nb=nb, target="d")
    sv = s.svd(A, U, VT, target="d")
    assert np.allclose(sv, np.linalg.svd(a, compute_uv=False), atol=1e-10 * n)
    u, vt = s.to_numpy(U), s.to_numpy(VT)
    assert np.linalg.norm(u @ np.diag(sv) @ vt - a) / (np.linalg.norm(a) * n) < 1e-12


@pytest.mark.parametrize("n,nb", [(1000, 64), (2500, 256)])
def test_bdsqr_device_vectors(n, nb):
    """Device bdsqr with both vector sets: the step-table rotation kernel
    (row counts not multiples of 64,
    several 16-sweep batches) against numpy's SVD of the bidiagonal."""
    rng = np.random.default_rng(41)
    d = rng.standard_normal(n)
    e = rng.standard_normal(n - 1)
    b = np.diag(d) + np.diag(e, 1)
    Ub = s.from_numpy(np.eye(n), nb=nb, target="d")
    VTb = s.from_numpy(np.eye(n), nb=nb, target="d")
    sig = np.asarray(s.bdsqr_matrix(s.Job.Vec, s.Job.Vec, d, e, Ub, VTb, target="d"))
    ref = np.linalg.svd(b, compute_uv=False)
    assert np.abs(np.sort(sig)[::-1] - ref).max() < 1e-12 * ref.max()
    u, vt = s.to_numpy(Ub), s.to_numpy(VTb)
    assert relerr((u * sig[None, :]) @ vt, b) < 1e-12
    assert np.linalg.norm(u.T @ u - np.eye(n)) / n < 1e-13
    assert np.linalg.norm(vt @ vt.T - np.eye(n)) / n < 1e-13


@pytest.mark.parametrize("kind", ["graded", "cluster", "toeplitz"])
def test_stedc_secular_device(kind):
    """Distributed stedc with the device secular-root kernel (rational
    two-pole iteration, secular.hh) on hard tridiagonals, against numpy."""
    n = 600
    if kind == "graded":
        d, e = np.logspace(0, -15, n), np.logspace(0, -15, n - 1) * 0.1
    elif kind == "cluster":
        d = np.ones(n)
        d[::7] = 1 + 1e-12
        e = np.full(n - 1, 1e-9)
    else:
        d, e = np.full(n, 2.0), np.full(n - 1, -1.0)
    t = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    tn = np.linalg.norm(t, 2)
    Q = s.from_numpy(np.zeros((n, n)), nb=64, target="d")
    w = np.asarray(s.stedc_matrix(d, e, Q, target="d"))
    z = s.to_numpy(Q)
    assert np.abs(np.sort(w) - np.linalg.eigvalsh(t)).max() <= 1e-13 * n * tn
    assert np.linalg.norm(t @ z - z * w) <= 1e-14 * n * tn
    assert np.linalg.norm(z.T @ z - np.eye(n)) <= 1e-14 * n


def test_condest_gmres_device():
    n, nb = 256, 64
    a = rnd(n, n, np.float64, 33) + n * np.eye(n)
    A = s.from_numpy(a, nb=nb, target="d")
    anorm = s.norm(s.Norm.One, A, target="d")
    info, _ = s.getrf(A, target="d")
    rc = s.gecondest(s.Norm.One, A, anorm, target="d")
    ref = 1 / np.linalg.cond(a, 1)
    assert ref * 0.999 <= rc <= 10 * ref
    b = rnd(n, 1, np.float64, 34)
    A2, B = s.from_numpy(a, nb=nb, target="d"), s.from_numpy(b, nb=nb, target="d")
    X = s.from_numpy(np.zeros_like(b), nb=nb, target="d")
    info, _, it = s.gesv_mixed_gmres(A2, B, X, target="d")
    assert info == 0 and it >= 0
    assert np.linalg.norm(a @ s.to_numpy(X) - b) / np.linalg.norm(b) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("thresh", [0.5, 0.1])
def test_getrf_pivot_threshold_device(thresh):
    """PivotThreshold in the device PPLU panel kernel (lu_pivot_kernel): |L| <= 1/threshold,
    P A = L U, and fewer interchanges than partial pivoting."""
    n, nb = 600, 128
    a = rnd(n, n, np.float64, 63) + 1.5 * np.eye(n)

    def run(**kw):
        A = s.from_numpy(a, nb=nb, target="d")
        info, piv = s.getrf(A, target="d", **kw)
        f = s.to_numpy(A)
        L = np.tril(f, -1) + np.eye(n)
        U = np.triu(f)
        ip = [kk * nb + ti * nb + off for kk, pv in enumerate(piv) for (ti, off) in pv]
        pa = a.copy()
        for j, p_ in enumerate(ip):
            pa[[j, p_]] = pa[[p_, j]]
        return info, relerr(L @ U, pa), np.abs(L).max(), sum(1 for j, p_ in enumerate(ip) if p_ != j)
    info, err, lmax, mv = run(pivot_threshold=thresh)
    _, _, _, mv1 = run()
    assert info == 0 and err < 1e-12 and lmax <= 1 / thresh + 1e-12 and mv < mv1


@pytest.mark.gpu
def test_hold_local_workspace_device():
    """Option::HoldLocalWorkspace (reference src/potrf.cc:42,198): a host-origin
    matrix factored on the device keeps its device copy only when held."""
    from slate_d35_amd import _slate
    n, nb = 512, 128
    a = rnd(n, n, np.float64, 64)
    a = a @ a.T + n * np.eye(n)
    for hold in (False, True):
        H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb))   # host origin
        before = _slate.bytes_in_use()
        assert s.potrf(H, target="d", hold_local_workspace=hold) == 0
        grown = _slate.bytes_in_use() - before
        assert (grown >= n * n * 8) == hold, (hold, grown)
        L = np.tril(s.to_numpy(H))
        assert relerr(L @ L.T, a) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_hesv_aasen_device(dtype):
    """Device-resident blocked Aasen (replicated T on the GPU, distributed panel
    LU, band LU of T) against numpy: indefinite Hermitian solve."""
    n, nb = 700, 64
    a = rnd(n, n, dtype, 71)
    h = (a + a.conj().T).astype(dtype)
    b = rnd(n, 4, dtype, 72)
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target="d"))
    T = s.BandMatrix(nb, nb, s.from_numpy(np.zeros((n, n), dtype), nb=nb, target="d"))
    B = s.from_numpy(b, nb=nb, target="d")
    info, p1, p2 = s.hesv_aasen(A, T, B, target="d")
    x = s.to_numpy(B)
    assert info == 0
    # backward error in the reference tester's form (test/test_hesv.cc:
    # ||b - A x|| / (||A|| ||x|| n) against a few eps); the band solve of T
    # runs on diagonal-block inverses + GEMMs, so allow 3 eps per row
    err = np.linalg.norm(h @ x - b) / (np.linalg.norm(h) * np.linalg.norm(x) * n)
    assert err < 3 * np.finfo(np.float64).eps, err


def test_band_storage_200k_fits_one_gpu():
    """Band-only storage at scale: n = 200000, kl = ku = 256 (dense would be
    320 GB) allocates O(n * bandwidth) and gbsv solves it on one GPU; checked
    through the band residual ||b - A x|| (gbmm over band chunks)."""
    n, kl, nb = 200000, 256, 256
    A = s.band_matrix(n, n, kl, kl, nb, target="d")
    assert A.is_band_storage and A.storage_bytes < 4 * 10**9, A.storage_bytes
    s._slate.generate_matrix_d("diag_dominant", A, 11, 4.0 * kl, s.opts("d"))
    b = rnd(n, 1, np.float64, 12)
    B = s.from_numpy(b, nb=nb, target="d")
    info, piv = s.gbsv(A, B, target="d")
    assert info == 0
    x = s.to_numpy(B)
    # residual with a fresh copy of the matrix (A holds the factors now)
    A0 = s.band_matrix(n, n, kl, kl, nb, target="d")
    s._slate.generate_matrix_d("diag_dominant", A0, 11, 4.0 * kl, s.opts("d"))
    R = s.from_numpy(b, nb=nb, target="d")
    s.gbmm(-1.0, A0, s.from_numpy(x, nb=nb, target="d"), 1.0, R, target="d")
    r = s.to_numpy(R)
    assert np.abs(r).max() / (s.norm(s.Norm.Inf, A0, target="d") * np.abs(x).max()) < 1e-13


@pytest.mark.parametrize("ranks", ["2", "4"])
def test_inproc_multirank_lapack_device(ranks):
    """Intra-process multi-GPU: ONE process runs the LAPACK shim's dgesv /
    dgetrf+dgetrs / dpotrf / dposv / dgemm on a grid of in-process ranks, each
    with its own device context (streams, allocator) and the peer-copy
    in-process communicator -- on this 1-GPU box all ranks share device 0."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SLATE_INPROC_RANKS=ranks, SLATE_LAPACK_TARGET="d", SLATE_LAPACK_NB="128")
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "inproc_check.py"), "1536"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "INPROC_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("variant", ["1", "2"])
def test_tournament_variants_all_types(variant):
    """Both tournament implementations (SLATE_TSLU=1: per-level launches, v1;
    2: one-launch tree + fused finish, v2) on every type, including the
    narrow last block (n = 100) and a three-level tree (complex: 256-row
    leaves, a node with fewer children than the fan-in).  The variant is read
    once per process, so each runs in its own interpreter."""
    import subprocess
    import sys
    code = r'''
import numpy as np, torch, sys
sys.path.insert(0, "ROOTDIR")
import slate_d35_amd as s
for dt in (np.float64, np.float32, np.complex128, np.complex64):
    for m, n in ((3000, 100), (9000, 64), (700, 96)):
        rng = np.random.default_rng(5)
        a = rng.uniform(-1, 1, (m, n))
        if np.iscomplexobj(np.zeros(1, dt)):
            a = a + 1j * rng.uniform(-1, 1, (m, n))
        a = a.astype(dt)
        tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
        info, ipiv = s.ops.getrf_panel(tA, tournament=True)
        f = tA.cpu().numpy().T
        k = min(m, n)
        L = np.tril(f[:, :k], -1) + np.eye(m, k)
        U = np.triu(f[:k, :])
        pa = a.copy()
        for j, p in enumerate(ipiv):
            pa[[j, p]] = pa[[p, j]]
        err = np.linalg.norm(L @ U - pa) / np.linalg.norm(pa)
        tol = 1e-4 if dt in (np.float32, np.complex64) else 1e-12
        assert info == 0 and err < tol and np.abs(L).max() < 8, (dt, m, n, info, err)
print("VARIANT_OK")
'''.replace("ROOTDIR", ROOT)
    env = dict(os.environ, SLATE_TSLU=variant)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "VARIANT_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_python_inproc_transparent():
    """A Python script on one process, no run_in_process: with
    SLATE_INPROC_RANKS=4 the device-target gesv / posv / gemm calls on a 1 x 1
    grid run on 2 x 2 in-process ranks (spread.hh); inproc_run_count() shows
    the path was taken and the residuals pass."""
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path.insert(0, "ROOTDIR")
import slate_d35_amd as s
n, nb = 1024, 128
rng = np.random.default_rng(3)
a = rng.uniform(-1, 1, (n, n)); b = rng.uniform(-1, 1, (n, 4))
A = s.from_numpy(a, nb=nb, target="d"); B = s.from_numpy(b, nb=nb, target="d")
c0 = s._slate.inproc_run_count()
info, piv = s.gesv(A, B, target="d")
x = s.to_numpy(B)
r1 = np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x) * n * 1e-16)
spd = a @ a.T + n * np.eye(n)
H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(spd, nb=nb, target="d")); B2 = s.from_numpy(b, nb=nb, target="d")
info2 = s.posv(H, B2, target="d")
x2 = s.to_numpy(B2)
r2 = np.linalg.norm(spd @ x2 - b) / (np.linalg.norm(spd) * np.linalg.norm(x2) * n * 1e-16)
C = s.from_numpy(np.zeros((n, n)), nb=nb, target="d")
s.gemm(1.0, s.from_numpy(a, nb=nb, target="d"), s.from_numpy(a.T.copy(), nb=nb, target="d"), 0.0, C, target="d")
r3 = np.abs(s.to_numpy(C) - a @ a.T).max()
runs = s._slate.inproc_run_count() - c0
print("RES", info, info2, r1, r2, r3, runs, s._slate.inproc_last_shape())
assert info == 0 and info2 == 0 and r1 < 50 and r2 < 50 and r3 < 1e-10 and runs >= 3, (r1, r2, r3, runs)
print("INPROC_OK")
'''.replace("ROOTDIR", ROOT)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(SLATE_INPROC_RANKS="4", SLATE_SPREAD_MIN_N="256", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "INPROC_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("nranks,count,rounds", [(3, 1000, 1), (4, 300000, 1), (5, 1 << 20, 1), (2, 300000, 1),
                                                  (4, 1 << 18, 12), (3, 3000, 8)])
def test_inproc_allreduce_device(nranks, count, rounds):
    """In-process all-reduce on device buffers: the all-to-all copy path for
    small messages and the reduce-scatter + all-gather path (>= 1 MiB, more
    than two ranks; uneven slices for 5 ranks).  rounds > 1: back-to-back
    all-reduce / bcast / all-reduce with skewed ranks (a fast rank enters the
    next collective while a slow one finishes the sliced hand-off)."""
    assert s._slate.inproc_allreduce_check(nranks, count, rounds) < 1e-12


# ---- multi-device matrices on the device (test_multi_device.py runs them in
# host mode on the CPU): the parts live in each in-process rank's device
# context -- four ranks on this box's one GPU -- and the drivers run on them
# in place (no scatter / gather per call, pinned by inproc_copy_bytes).
def test_multi_device_lu_on_device():
    import test_multi_device as md
    md.test_lu_factor_then_solve_twice_no_copies(np.float64)


def test_multi_device_cholesky_blas_on_device():
    import test_multi_device as md
    md.test_cholesky_and_trsm_herk_gemm()


def test_multi_device_qr_on_device():
    import test_multi_device as md
    md.test_qr_least_squares_and_unmqr()


def test_multi_device_mixed_eig_on_device():
    import test_multi_device as md
    md.test_mixed_precision_and_eig_svd()


def test_multi_device_layout_on_device():
    import test_multi_device as md
    md.test_multi_device_layout_and_gather()
    A = s.multi_device(300, 300, 64, np.float64, 4)
    assert A.is_multi_device and A.num_parts == 4


def test_from_devices_device_arrays():
    """fromDevices(Aarray, num_devices) over device arrays (torch tensors on
    this GPU standing in for per-GPU arrays: 1 x 3 in-process ranks)."""
    torch = _torch()
    m, n, nb, nd = 200, 170, 32, 3
    a = np.random.default_rng(3).standard_normal((m, n))
    nt = -(-n // nb)
    cols = [[j for j in range(nt) if j % nd == d] for d in range(nd)]
    idx = [np.concatenate([np.arange(j * nb, min(n, (j + 1) * nb)) for j in c]) for c in cols]
    if torch.cuda.device_count() >= nd:
        pytest.skip("one-GPU layout check (several GPUs: device d must hold array d)")
    ts = [torch.tensor(np.ascontiguousarray(a[:, ix].T), device="cuda") for ix in idx]   # column-major m x k
    torch.cuda.synchronize()
    A = s.from_devices(m, n, [t.data_ptr() for t in ts], m, nb)
    assert A.is_multi_device and A.num_parts == nd
    assert np.array_equal(s.to_numpy(A), a)
    s.scale(2.0, 1.0, A)                         # in place, in the caller's arrays
    torch.cuda.synchronize()
    assert np.array_equal(ts[1].cpu().numpy().T, 2 * a[:, idx[1]])
