"""C++ examples (reference examples/ex01-ex15 + examples/run_tests.py): every
example on 1 process, and the distributed ones on 2 and 4 processes over the
native TCP transport (the C++ programs bootstrap with slate::init_grid from
the torchrun-style environment; no Python in the ranks).  Host target here;
the GPU variant runs the same binaries with SLATE_TARGET=d."""
import glob
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin")
EXAMPLES = sorted(os.path.basename(p)[:-3] for p in glob.glob(os.path.join(ROOT, "examples", "cpp", "ex*.cc")))
MULTI = ["ex01_matrix", "ex04_norm", "ex05_blas", "ex06_linear_system_lu", "ex07_linear_system_cholesky",
         "ex09_least_squares", "ex11_hermitian_eig", "ex13_redistribute", "ex14_scalapack_gemm", "ex15_set_matrix"]


@pytest.fixture(scope="module", autouse=True)
def built():
    r = subprocess.run(["make", "-j8", "examples"], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(exe, nprocs, target="h", timeout=300):
    port = _port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SLATE_MASTER_PORT=str(port), SLATE_TARGET=target, SLATE_COMM="host",
                   OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([os.path.join(BIN, exe)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    codes = [p.returncode for p in procs]
    return codes, outs


@pytest.mark.parametrize("exe", EXAMPLES)
def test_example_single_process(exe):
    codes, outs = launch(exe, 1)
    assert codes == [0] and "all passed" in outs[0], outs[0][-3000:]


@pytest.mark.parametrize("nprocs", [2, 4])
@pytest.mark.parametrize("exe", MULTI)
def test_example_multi_process(exe, nprocs):
    codes, outs = launch(exe, nprocs)
    assert codes == [0] * nprocs and "all passed" in outs[0], "\n".join(o[-1500:] for o in outs)


@pytest.mark.gpu
@pytest.mark.parametrize("exe", ["ex05_blas", "ex06_linear_system_lu", "ex07_linear_system_cholesky",
                                 "ex10_svd", "ex11_hermitian_eig"])
def test_example_device(exe):
    codes, outs = launch(exe, 1, target="d")
    assert codes == [0] and "all passed" in outs[0], outs[0][-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("exe", ["ex05_blas", "ex06_linear_system_lu", "ex07_linear_system_cholesky"])
def test_example_inproc_transparent(exe):
    """One process, several GPUs, no explicit run_in_process: the unchanged
    examples (1 x 1 grid, Target::Devices) with SLATE_INPROC_RANKS=4 run
    gemm / getrf / getrs / gesv / potrf / potrs / posv on a 2 x 2 grid of
    in-process ranks (csrc/src/spread.hh; 4 ranks on the box's one GPU here)
    and pass their residual checks.  The example reports the number of
    driver calls that took the in-process path."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env.update(SLATE_TARGET="d", SLATE_INPROC_RANKS="4", SLATE_SPREAD_MIN_N="256", OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(BIN, exe)], env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "all passed" in out, out[-3000:]
    assert "in-process multi-GPU driver runs:" in out and "last grid 2 x 2" in out, out[-3000:]
