"""Stage timings of heev / svd on one process (trace blocks summed by name).

usage: python scripts/eig_prof.py N [NB] [target] [routines]
"""
import os
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: F401,E402
import slate_d35_amd as s  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 256
tg = sys.argv[3] if len(sys.argv) > 3 else "d"
routines = (sys.argv[4] if len(sys.argv) > 4 else "heev,svd").split(",")
out = os.environ.get("EIG_PROF_OUT", "gpurun_out")
os.makedirs(out, exist_ok=True)
rng = np.random.default_rng(1)
a = rng.standard_normal((n, n))
h = a + a.T


def stages():
    tot = defaultdict(float)
    for name, t0, t1, lane in s.trace.events():
        if lane < 100:              # host blocks only
            tot[name] += (t1 - t0) * 1e3
    return dict(sorted(tot.items(), key=lambda kv: -kv[1]))


for r in routines:
    for step in range(2):
        if r == "heev":
            A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
            Z = s.from_numpy(np.zeros((n, n)), nb=nb, target=tg)
        else:
            A = s.from_numpy(a, nb=nb, target=tg)
            U = s.from_numpy(np.zeros((n, n)), nb=nb, target=tg)
            VT = s.from_numpy(np.zeros((n, n)), nb=nb, target=tg)
        if step == 1:
            s.trace.on()
        t0 = time.perf_counter()
        if r == "heev":
            lam = s.heev(A, Z, target=tg)
        else:
            sv = s.svd(A, U, VT, target=tg)
        dt = time.perf_counter() - t0
        if step == 1:
            st = stages()
            s.trace.off()
            s.trace.clear()
            flops = (4.0 / 3.0 + 4.0) * n ** 3 if r == "heev" else 22.0 * n ** 3   # LAPACK-style op counts
            print(f"{r} n={n} nb={nb} {tg}: {dt:.3f} s  ({flops / dt / 1e9:.1f} GF/s nominal)", flush=True)
            for k, v in list(st.items())[:30]:
                print(f"    {k:28s} {v:10.1f} ms", flush=True)
    if r == "heev":
        zz = s.to_numpy(Z)
        res = np.linalg.norm(h @ zz - zz * lam) / (np.linalg.norm(h) * n)
        print(f"    residual {res:.2e}", flush=True)
