#!/usr/bin/env python3
"""Run N ranks of the native tester on ONE GPU over the real RCCL transport.
RCCL refuses two ranks of one communicator on the same device of the same
host; giving every rank its own NCCL_HOSTID makes them distinct "hosts", so
RCCL connects them through its socket transport over loopback.  This is a
test rig for the RCCL code path only (bandwidth is meaningless).
Usage: rccl_multi.py NPROCS tester-args...   |   rccl_multi.py NPROCS --cmd prog args..."""
import os, socket, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1])
args = sys.argv[2:]
cmd = args[1:] if args and args[0] == "--cmd" else [os.path.join(ROOT, "bin", "slate_tester")] + args
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
env0 = {k: v for k, v in os.environ.items() if k != "SLATE_COMM"}
procs = []
# every rank writes straight to its own file (progress stays visible during long runs)
logdir = os.environ.get("RANK_LOGDIR", os.path.join(ROOT, "gpurun_out", "ranks"))
os.makedirs(logdir, exist_ok=True)
files = [open(os.path.join(logdir, f"rank{r}.log"), "w+") for r in range(n)]
for r in range(n):
    env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), SLATE_MASTER_PORT=str(port), NCCL_HOSTID=f"slate-fake-host-{r}",
               NCCL_SOCKET_IFNAME="lo", NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"), OMP_NUM_THREADS="2")
    # RANK0_WRAP: a prefix for rank 0's command only, e.g. a profiler
    # ("rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o r0 --"): the
    # profiled program is the tester itself, started from this launcher
    wrap = os.environ.get("RANK0_WRAP", "").split() if r == 0 else []
    procs.append(subprocess.Popen(wrap + cmd, stdout=files[r], stderr=subprocess.STDOUT, text=True, env=env))
outs, codes = [], []
try:
    for r, p in enumerate(procs):
        p.wait(timeout=int(os.environ.get("RANK_TIMEOUT", "300")))
        codes.append(p.returncode)
        files[r].seek(0)
        outs.append(files[r].read())
finally:
    for p in procs:
        if p.poll() is None:
            p.kill()
for r, o in enumerate(outs):
    print(f"===== rank {r} rc={codes[r]}")
    print(o[-6000:] if r == 0 else o[-1500:])
sys.exit(0 if all(c == 0 for c in codes) else 1)
