"""bench.py contract (host target, small n): one JSON line with the
BASELINE metric, and the fail-fast watchdog that turns a hung step into
exit code 124 instead of a run that holds the node until the driver's limit."""
import json
import os
import subprocess
import sys

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
