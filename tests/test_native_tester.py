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
    assert outs[0].count("pass") >= 40


@pytest.mark.parametrize("nprocs,grid", [(2, "1x2"), (4, "2x2")])
def test_distributed_subset(nprocs, grid):
    codes, outs = launch(["gemm,herk,trsm,potrf,getrf,getrf_tntpiv,geqrf,gels,gesv_mixed,heev", "--type", "d",
                          "--dim", "192", "--nb", "32", "--grid", grid], nprocs)
    assert codes == [0] * nprocs and "all tests passed" in outs[0], "\n".join(o[-2500:] for o in outs)


def test_rectangular_and_sweeps():
    codes, outs = launch(["gemm,geqrf,gelqf,gels", "--type", "s,d", "--dim", "150x90x60,90x150x60", "--nb", "32,40"])
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]


@pytest.mark.gpu
def test_device_routines():
    codes, outs = launch(["gemm,herk,trsm,potrf,getrf,getrf_tntpiv,geqrf,gesv_mixed,posv_mixed,heev,svd",
                          "--type", "d,z", "--dim", "1000", "--nb", "128"], target="d")
    assert codes == [0] and "all tests passed" in outs[0], outs[0][-4000:]
