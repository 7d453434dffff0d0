"""bench.py contract (host target, small n): one JSON line with the
BASELINE metric, and the fail-fast watchdog that turns a hung step into
exit code 124 instead of a run that holds the node until the driver's limit."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_json_line():
    r = _bench(["--dim", "512", "--nb", "128", "--steps", "1", "--warmup", "0", "--extras", "none"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert line["metric"] == base["metric"] and line["n_gpus"] == 1 and line["steps"] == 1
    assert set(line["routines"]) == {"dgemm", "dpotrf", "dgetrf", "dgeqrf"}
    assert all(v["check"] == "pass" for v in line["routines"].values())


def test_bench_watchdog_exits_124():
    r = _bench(["--dim", "4096", "--routines", "dgeqrf", "--steps", "1", "--warmup", "0", "--extras", "none",
                "--check", "no"], env_extra={"SLATE_BENCH_STEP_TIMEOUT": "1"})
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert "WATCHDOG rank 0: 'dgeqrf step 0'" in r.stderr


def _last_json(out):
    return json.loads([ln for ln in out.strip().splitlines() if ln.startswith("{")][-1])


def test_bench_self_launch_4_ranks():
    """`python3 bench.py --gpus 4` with no launcher environment spawns its own
    four rank processes (host target here); the JSON reports what the
    communicators that were actually created saw."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dim", "1024", "--nb", "128",
                        "--steps", "1", "--warmup", "0", "--extras", "none"], env=dict(env, OMP_NUM_THREADS="2"),
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 4
    comm = line["config"]["comm"]
    assert comm["world"] == 4 and comm["row"] * comm["col"] == 4 and comm["grid"] == [2, 2]
    assert comm["launcher"] == "self" and len(comm["devices"]) == 4
    assert all(v["check"] == "pass" for v in line["routines"].values())
    # per-routine grids of the 4-GPU defaults (bench.GRID_PER, from the
    # critical-path sweep): QR and Cholesky on 4 x 1, the rest on the job's 2 x 2
    grids = {k: v["grid"] for k, v in line["routines"].items()}
    assert grids == {"dgemm": "2x2", "dpotrf": "4x1", "dgetrf": "2x2", "dgeqrf": "4x1"}, grids


def test_bench_self_launch_propagates_failure():
    """A rank that fails (here: its watchdog fires) makes the launcher exit
    with that rank's code and stop the other ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SLATE_BENCH_STEP_TIMEOUT="1", OMP_NUM_THREADS="2", SLATE_BENCH_RANK_GRACE="20")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dim", "4096",
                        "--routines", "dgeqrf", "--steps", "1", "--warmup", "0", "--extras", "none", "--check", "no"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert "WATCHDOG" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8])
def test_bench_self_launch_rccl_one_gpu(n):
    """`bench.py --gpus N` launched with no torchrun on the one-GPU box: N
    rank processes, each with its own NCCL_HOSTID (SLATE_BENCH_FAKE_HOSTS) so
    RCCL forms real N-rank communicators on one device.  Asserts the
    communicator sizes RCCL reports and the residual checks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SLATE_COMM")}
    env.update(SLATE_BENCH_FAKE_HOSTS="1", OMP_NUM_THREADS="2", NCCL_DEBUG="WARN")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dim", "4096",
                        "--nb", "256", "--steps", "1", "--warmup", "0", "--extras", "none"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    line = _last_json(r.stdout)
    comm = line["config"]["comm"]
    assert line["n_gpus"] == n and comm["backend"] == "rccl" and comm["world"] == n
    assert comm["row"] * comm["col"] == n and comm["devices"] == [0] * n
    assert all(v["check"] == "pass" for v in line["routines"].values())
