"""Time the device panel factorizations in isolation (no concurrent trailing
update): getrf_panel (partial / tournament) and geqrf_panel on m x nb."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import slate_d35_amd as s

m = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 512
reps = 5
torch.manual_seed(0)
A0 = torch.rand(nb, m, dtype=getattr(torch, os.environ.get("DTYPE", "float64")), device="cuda") * 2 - 1   # column-major m x nb
ONLY = os.environ.get("PANELS", "")
for name, fn in [("getrf_partial", lambda A: s.ops.getrf_panel(A, tournament=False)),
                 ("getrf_tournament", lambda A: s.ops.getrf_panel(A, tournament=True)),
                 ("geqrf", lambda A: s.ops.geqrf_panel(A))]:
    if ONLY and not any(o in name for o in ONLY.split(",")):
        continue
    ts = []
    for r in range(reps + 1):
        A = A0.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(A)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts[1:])
    print(f"{name:18s} m={m} nb={nb}: {t*1e3:8.2f} ms", flush=True)
