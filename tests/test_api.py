"""C / Fortran / LAPACK-compatible / ScaLAPACK-compatible APIs (reference
test strategy: lapack_api/example_dgetrf.c, scalapack_api/example_pdgetrf.c,
examples/c_api).  LAPACK/ScaLAPACK symbols are called through ctypes with
Fortran conventions (everything by reference)."""
import ctypes as C
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import slate_d35_amd as s  # noqa: F401  (loads libslate_amd)
from helpers import rnd, relerr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slate_d35_amd")
ENV = dict(os.environ, SLATE_LAPACK_TARGET="h", SLATE_SCALAPACK_TARGET="h")


@pytest.fixture(scope="module")
def lapack():
    os.environ["SLATE_LAPACK_TARGET"] = "h"
    return C.CDLL(os.path.join(PKG, "libslate_lapack_api.so"))


@pytest.fixture(scope="module")
def scalapack():
    os.environ["SLATE_SCALAPACK_TARGET"] = "h"
    return C.CDLL(os.path.join(PKG, "libslate_scalapack_api.so"))


def I(v):
    return C.byref(C.c_int(v))


def ch(c):
    return C.c_char_p(c.encode())


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


@pytest.mark.parametrize("nprocs", [1, 2, 4])
def test_c_api_grid_example(tmp_path, nprocs):
    """C program on a p x q grid bootstrapped by slate_grid_init from the
    torchrun-style environment (native TCP transport here)."""
    import socket
    exe = tmp_path / "ex_c_api_grid"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT}/csrc/include", f"{ROOT}/examples/ex_c_api_grid.c", f"-L{PKG}",
                    "-lslate_amd", f"-Wl,-rpath,{PKG}", "-lm", "-o", str(exe)], check=True)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=dict(ENV, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SLATE_MASTER_PORT=str(port),
                                       SLATE_COMM="host", OMP_NUM_THREADS="2"))
             for r in range(nprocs)]
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(outs)
    assert "info=0" in outs[0] and f"{nprocs} ranks" in outs[0]


def test_c_api_example(tmp_path):
    exe = tmp_path / "ex_c_api"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT}/csrc/include", f"{ROOT}/examples/ex_c_api.c", f"-L{PKG}",
                    "-lslate_amd", f"-Wl,-rpath,{PKG}", "-lm", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "info=0" in r.stdout


@pytest.mark.skipif(shutil.which("amdflang") is None and not os.path.exists("/opt/rocm/bin/amdflang"),
                    reason="no Fortran compiler")
def test_fortran_example(tmp_path):
    fc = shutil.which("amdflang") or "/opt/rocm/bin/amdflang"
    subprocess.run([fc, "-c", f"{ROOT}/csrc/api/slate_c_api.f90", "-module-dir", str(tmp_path), "-o",
                    str(tmp_path / "m.o")], check=True)
    exe = tmp_path / "ex_f"
    subprocess.run([fc, f"-I{tmp_path}", f"{ROOT}/examples/ex_fortran.f90", str(tmp_path / "m.o"), f"-L{PKG}",
                    "-lslate_amd", f"-Wl,-rpath,{PKG}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_fortran_module_generated(tmp_path):
    """The checked-in Fortran module matches the generator's output for c_api.h
    (every C API function has an interface, all four precisions)."""
    out = tmp_path / "gen.f90"
    subprocess.run([sys.executable, f"{ROOT}/csrc/api/gen_fortran.py", str(out)], check=True, capture_output=True)
    assert out.read_text() == open(f"{ROOT}/csrc/api/slate_c_api.f90").read()
    assert out.read_text().count("bind(c, name=") >= 200


def test_lapack_gesv_gemm_potrf(lapack):
    n, nrhs = 150, 3
    a = np.asfortranarray(rnd(n, n, np.float64, 1))
    b = np.asfortranarray(rnd(n, nrhs, np.float64, 2))
    a0, b0 = a.copy(), b.copy()
    ipiv = np.zeros(n, np.int32)
    info = C.c_int(0)
    lapack.slate_dgesv_(I(n), I(nrhs), ptr(a), I(n), ptr(ipiv), ptr(b), I(n), C.byref(info))
    assert info.value == 0
    assert relerr(a0 @ b, b0) < 1e-12
    # pivots are LAPACK-style 1-based
    assert ipiv.min() >= 1 and ipiv.max() <= n
    # getrs with the returned factors, transposed system
    x = np.asfortranarray(b0.copy())
    lapack.slate_dgetrs_(ch("T"), I(n), I(nrhs), ptr(a), I(n), ptr(ipiv), ptr(x), I(n), C.byref(info))
    assert relerr(a0.T @ x, b0) < 1e-12
    # gemm
    m, k = 70, 40
    A = np.asfortranarray(rnd(k, m, np.float64, 3))
    B = np.asfortranarray(rnd(k, n, np.float64, 4))
    Cm = np.asfortranarray(rnd(m, n, np.float64, 5))
    c0 = Cm.copy()
    al, be = C.c_double(2.0), C.c_double(-1.0)
    lapack.slate_dgemm_(ch("T"), ch("N"), I(m), I(n), I(k), C.byref(al), ptr(A), I(k), ptr(B), I(k), C.byref(be),
                        ptr(Cm), I(m))
    assert relerr(Cm, 2.0 * A.T @ B - c0) < 1e-13
    # potrf
    spd = np.asfortranarray(a0 @ a0.T + n * np.eye(n))
    s0 = spd.copy()
    lapack.slate_dpotrf_(ch("L"), I(n), ptr(spd), I(n), C.byref(info))
    L = np.tril(spd)
    assert info.value == 0 and relerr(L @ L.T, s0) < 1e-13
    lapack.slate_dlange_.restype = C.c_double
    w = np.zeros(1)
    assert abs(lapack.slate_dlange_(ch("F"), I(n), I(n), ptr(a0), I(n), ptr(w)) - np.linalg.norm(a0)) < 1e-9


def test_lapack_syev_gesvd_complex(lapack):
    n = 80
    h = rnd(n, n, np.float64, 6)
    h = np.asfortranarray(h + h.T)
    h0 = h.copy()
    wv = np.zeros(n)
    info = C.c_int(0)
    work = np.zeros(1)
    lapack.slate_dsyev_(ch("V"), ch("L"), I(n), ptr(h), I(n), ptr(wv), ptr(work), I(1), C.byref(info))
    assert np.allclose(wv, np.linalg.eigvalsh(h0), atol=1e-10)
    assert np.linalg.norm(h0 @ h - h * wv) < 1e-9
    m = 90
    g = np.asfortranarray(rnd(m, n, np.float64, 7))
    g0 = g.copy()
    sv = np.zeros(n)
    U = np.zeros((m, n), order="F")
    VT = np.zeros((n, n), order="F")
    lapack.slate_dgesvd_(ch("S"), ch("S"), I(m), I(n), ptr(g), I(m), ptr(sv), ptr(U), I(m), ptr(VT), I(n),
                         ptr(work), I(1), C.byref(info))
    assert info.value == 0 and relerr(U @ np.diag(sv) @ VT, g0) < 1e-12
    z = np.asfortranarray(rnd(60, 60, np.complex128, 8))
    z0 = z.copy()
    ipiv = np.zeros(60, np.int32)
    lapack.slate_zgetrf_(I(60), I(60), ptr(z), I(60), ptr(ipiv), C.byref(info))
    bz = np.asfortranarray(rnd(60, 1, np.complex128, 9))
    bz0 = bz.copy()
    lapack.slate_zgetrs_(ch("N"), I(60), I(1), ptr(z), I(60), ptr(ipiv), ptr(bz), I(60), C.byref(info))
    assert relerr(z0 @ bz, bz0) < 1e-12


def desc(m, n, mb, nb, lld):
    return np.array([1, 0, m, n, mb, nb, 0, 0, lld], dtype=np.int32)


def test_scalapack_pdgemm_pdgesv_pdposv(scalapack):
    n, nb = 128, 32
    a = np.asfortranarray(rnd(n, n, np.float64, 10)) + n * np.eye(n, order="F")
    b = np.asfortranarray(rnd(n, 2, np.float64, 11))
    a0, b0 = a.copy(), b.copy()
    da, db = desc(n, n, nb, nb, n), desc(n, 2, nb, nb, n)
    ipiv = np.zeros(n + nb, np.int32)
    info = C.c_int(0)
    scalapack.pdgesv_(I(n), I(2), ptr(a), I(1), I(1), ptr(da), ptr(ipiv), ptr(b), I(1), I(1), ptr(db),
                      C.byref(info))
    assert info.value == 0 and relerr(a0 @ b, b0) < 1e-12
    # pdgemm on a tile-aligned sub-matrix: C(33:96, 33:96) = A(33:96, 1:64) B(1:64, 33:96)
    A = np.asfortranarray(rnd(n, n, np.float64, 12))
    B = np.asfortranarray(rnd(n, n, np.float64, 13))
    Cm = np.zeros((n, n), order="F")
    d = desc(n, n, nb, nb, n)
    al, be = C.c_double(1.0), C.c_double(0.0)
    scalapack.PDGEMM(ch("N"), ch("N"), I(64), I(64), I(64), C.byref(al), ptr(A), I(33), I(1), ptr(d),
                     ptr(B), I(1), I(33), ptr(d), C.byref(be), ptr(Cm), I(33), I(33), ptr(d))
    assert relerr(Cm[32:96, 32:96], A[32:96, 0:64] @ B[0:64, 32:96]) < 1e-13
    spd = np.asfortranarray(a0 @ a0.T)
    s0 = spd.copy()
    bb = np.asfortranarray(b0.copy())
    scalapack.pdposv_(ch("U"), I(n), I(2), ptr(spd), I(1), I(1), ptr(da), ptr(bb), I(1), I(1), ptr(db),
                      C.byref(info))
    assert info.value == 0 and relerr(s0 @ bb, b0) < 1e-10


def test_scalapack_pdsgesv_pzcgesv(scalapack):
    """p?gesv_mixed (reference scalapack_api/scalapack_gesv_mixed.cc): fp32
    factor, fp64 refinement; A keeps its fp64 values, X the refined solution."""
    n, nb = 96, 32
    for dt, fn in ((np.float64, scalapack.pdsgesv_), (np.complex128, scalapack.pzcgesv_)):
        a = np.asfortranarray(rnd(n, n, dt, 21)) + n * np.eye(n, order="F")
        b = np.asfortranarray(rnd(n, 3, dt, 22))
        x = np.zeros((n, 3), dtype=dt, order="F")
        a0, b0 = a.copy(), b.copy()
        da, db = desc(n, n, nb, nb, n), desc(n, 3, nb, nb, n)
        ipiv = np.zeros(n + nb, np.int32)
        it, info = C.c_int(0), C.c_int(0)
        fn(I(n), I(3), ptr(a), I(1), I(1), ptr(da), ptr(ipiv), ptr(b), I(1), I(1), ptr(db),
           ptr(x), I(1), I(1), ptr(db), C.byref(it), C.byref(info))
        assert info.value == 0 and it.value >= 0
        assert relerr(a0 @ x, b0) < 1e-12
        assert np.array_equal(b, b0)


def _inproc_lapack_case(lapack, dt, pre):
    """slate_?gesv_ / ?getrf_ + ?getrs_ / ?potrf_ / ?posv_ / ?gemm_ of ONE
    process on a grid of in-process ranks (inproc.hh; host mode here, one
    rank per GPU on a GPU box)."""
    n, nb = 200, 32
    f = lambda name: getattr(lapack, f"slate_{pre}{name}_")
    a = np.asfortranarray(rnd(n, n, dt, 61)) + n * np.eye(n, order="F")
    b = np.asfortranarray(rnd(n, 3, dt, 62))
    a0, b0 = a.copy(), b.copy()
    ipiv = np.zeros(n, np.int32)
    info = C.c_int(-7)
    f("gesv")(I(n), I(3), ptr(a), I(n), ptr(ipiv), ptr(b), I(n), C.byref(info))
    assert info.value == 0 and relerr(a0 @ b, b0) < 1e-12
    # getrf + getrs, ipiv in LAPACK convention
    a = a0.copy(order="F")
    f("getrf")(I(n), I(n), ptr(a), I(n), ptr(ipiv), C.byref(info))
    assert info.value == 0
    L = np.tril(a, -1) + np.eye(n)
    U = np.triu(a)
    pa = a0.copy()
    for i, pv in enumerate(ipiv):
        pa[[i, pv - 1]] = pa[[pv - 1, i]]
    assert relerr(L @ U, pa) < 1e-12
    bb = b0.copy(order="F")
    f("getrs")(ch("N"), I(n), I(3), ptr(a), I(n), ptr(ipiv), ptr(bb), I(n), C.byref(info))
    assert relerr(a0 @ bb, b0) < 1e-12
    # Cholesky
    h = np.asfortranarray(a0 @ a0.conj().T)
    h0 = h.copy()
    f("potrf")(ch("L"), I(n), ptr(h), I(n), C.byref(info))
    Lc = np.tril(h)
    assert info.value == 0 and relerr(Lc @ Lc.conj().T, h0) < 1e-12
    h = h0.copy(order="F")
    bb = b0.copy(order="F")
    f("posv")(ch("U"), I(n), I(3), ptr(h), I(n), ptr(bb), I(n), C.byref(info))
    assert info.value == 0 and relerr(h0 @ bb, b0) < 1e-10
    # gemm with transposes
    g1 = np.asfortranarray(rnd(150, n, dt, 63))
    g2 = np.asfortranarray(rnd(n, 90, dt, 64))
    c = np.asfortranarray(rnd(n, 90, dt, 65))
    c0 = c.copy()
    one = (C.c_double * 2)(1.0, 0.0) if dt == np.complex128 else C.c_double(1.0)
    half = (C.c_double * 2)(0.5, 0.0) if dt == np.complex128 else C.c_double(0.5)
    f("gemm")(ch("T"), ch("N"), I(n), I(90), I(150), C.byref(one), ptr(g1), I(150), ptr(g2[:150].copy(order="F")),
              I(150), C.byref(half), ptr(c), I(n), )
    assert relerr(c, g1.T @ g2[:150] + 0.5 * c0) < 1e-13


@pytest.mark.parametrize("ranks", ["2", "4", "8"])
def test_lapack_inproc_ranks(lapack, ranks, monkeypatch):
    monkeypatch.setenv("SLATE_INPROC_RANKS", ranks)
    monkeypatch.setenv("SLATE_LAPACK_NB", "32")
    c0 = s._slate.inproc_run_count()
    for dt, pre in ((np.float64, "d"), (np.complex128, "z")):
        _inproc_lapack_case(lapack, dt, pre)
    # every call above took the multi-rank path: 6 per type
    assert s._slate.inproc_run_count() - c0 == 12
    p, q = s._slate.inproc_last_shape()
    assert p * q == int(ranks) and p <= q
