"""Native C++ tester (reference test/tester + run_tests.py): every routine on
the host target, and a subset on 2 / 4 processes over the native transport;
the checks are the tester's own distributed backward-error residuals."""
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "bin", "slate_tester")


@pytest.fixture(scope="module", autouse=True)
def built():
    r = subprocess.run(["make", "tester"], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def launch(args, nprocs=1, timeout=600, target="h"):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([EXE] + args + ["--target", target], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True, env=dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                                                  MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                                                  SLATE_MASTER_PORT=str(port), SLATE_COMM="host",
                                                  OMP_NUM_THREADS="2"))
             for r in range(nprocs)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [p.returncode for p in procs], outs


def test_all_routines_single_process():
    codes, outs = launch(["all", "--type", "d,z", "--dim", "200", "--nb", "48"])
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]
    assert outs[0].count("pass") >= 180       # ~100 routines x 2 types (real-only ones skip for z)


@pytest.mark.parametrize("nprocs,grid", [(2, "1x2"), (4, "2x2")])
def test_distributed_subset(nprocs, grid):
    codes, outs = launch(["gemm,herk,trsm,potrf,getrf,getrf_tntpiv,geqrf,gels,gesv_mixed,heev", "--type", "d",
                          "--dim", "192", "--nb", "32", "--grid", grid], nprocs)
    assert codes == [0] * nprocs and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)


def test_rectangular_and_sweeps():
    codes, outs = launch(["gemm,geqrf,gelqf,gels", "--type", "s,d", "--dim", "150x90x60,90x150x60", "--nb", "32,40"])
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]


def test_breadth_distributed_2x2():
    """The breadth additions (rank-2k, stationary-A, condest, unm*, cholqr,
    band, indefinite, generalized eig, tridiagonal, aux) on a 2x2 grid."""
    codes, outs = launch(["syrk,her2k,syr2k,symm,gemmA,gemmC,getrs,potrs,potri,gesv_nopiv,gesv_tntpiv,gesv_rbt,"
                          "gecondest,pocondest,unmqr,unmlq,cholqr,gbtrf,pbsv,gbmm,hbmm,tbsm,tbsm_pivots,hetrf,heev_vals,svd_vals,"
                          "hegv,steqr2,add,copy,scale,set,trtrm,colnorms,henorm,redistribute",
                          "--type", "d,z", "--dim", "150", "--nb", "32", "--grid", "2x2"], 4)
    assert codes == [0] * 4 and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)


def test_tester_flags():
    """--matrix (element and spectral matgen kinds), --method-lu/trsm/gemm,
    --origin h, --timer-level 2 (per-driver times), --pivot-threshold."""
    codes, outs = launch(["getrf,gesv,trsm,gemm,geqrf", "--type", "d", "--dim", "160", "--nb", "32", "--matrix", "svd",
                          "--method-lu", "calu", "--method-trsm", "A", "--method-gemm", "A", "--origin", "h",
                          "--timer-level", "2", "--pivot-threshold", "0.5"])
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]
    assert "#   getrf" in outs[0]


def test_breadth2_distributed_2x2():
    """Stage-level eigen/SVD routines, the remaining solve variants, band /
    symmetric / triangular norms, trapezoid aux variants and sy* solvers on a
    2x2 grid (reference test/test.cc routine list)."""
    codes, outs = launch(["he2hb,unmtr_he2hb,hb2st,unmtr_hb2st,ge2tb,tb2bd,unmbr_tb2bd,bdsqr,stedc,hegst,"
                          "getrs_nopiv,getrs_tntpiv,posv_mixed_gmres,gbtrs,pbtrs,scale_row_col,gbnorm,hbnorm,synorm,"
                          "trnorm,tzset,tzcopy,tzscale,tzadd,sysv,sytrf,sytrs,hetrs,stedc_z_vector,stedc_sort,"
                          "stedc_deflate,stedc_secular",
                          "--type", "d,z", "--dim", "150,140x110x110", "--nb", "32", "--grid", "2x2"], 4)
    assert codes == [0] * 4 and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)


@pytest.mark.parametrize("flags", [["--side", "r", "--trans", "c", "--uplo", "u", "--diag", "u"],
                                   ["--side", "l", "--trans", "t", "--uplo", "u"]])
def test_shape_flags(flags):
    """--side / --trans / --uplo / --diag on the triangular routines and norms."""
    codes, outs = launch(["trsm,trmm,trnorm,synorm,tzset,tzadd", "--type", "d,z", "--dim", "130x90x90", "--nb", "32"]
                         + flags)
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]


def test_nonuniform_and_grid_order():
    """--nonuniform-nb y (alternating nb, nb/2+1 tiles on a 2-D cyclic map:
    the drivers' arbitrary-layout path), --go r (row-major process grid),
    --cond with a spectral --matrix, --ib."""
    codes, outs = launch(["getrf,gesv,geqrf,gels,heev", "--type", "d", "--dim", "170x130x130,160", "--nb", "32",
                          "--grid", "1x2", "--nonuniform-nb", "y", "--go", "r", "--ib", "16"], 2)
    assert codes == [0, 0] and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)
    codes, outs = launch(["gesv,getrf", "--type", "d", "--dim", "200", "--nb", "32", "--matrix", "svd", "--cond", "1e6"])
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]


@pytest.mark.gpu
def test_device_routines():
    codes, outs = launch(["gemm,herk,trsm,potrf,getrf,getrf_tntpiv,geqrf,gesv_mixed,posv_mixed,heev,svd,"
                          "syr2k,symm,gemmA,getrs,potri,gesv_rbt,unmqr,unmlq,cholqr,gbtrf,pbsv,hbmm,tbsm,tbsm_pivots,heev_vals,"
                          "svd_vals,hegv,steqr2,redistribute",
                          "--type", "d,z", "--dim", "1000", "--nb", "128"], target="d")
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]


@pytest.mark.parametrize("method", ["herkC", "gemmA", "gemmC"])
def test_cholqr_methods(method):
    """--method-cholqr: A^H A by herk (triangle), stationary-A gemm or SUMMA
    gemm (reference method.hh MethodCholQR), on a 2x2 grid."""
    codes, outs = launch(["cholqr", "--type", "d,z", "--dim", "170x90x90", "--nb", "32", "--grid", "2x2",
                          "--method-cholqr", method], 4)
    assert codes == [0] * 4 and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)
