"""Step through ge2tb on host and device, comparing the matrix after each op."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch  # noqa
import slate_d35_amd as s
from helpers import rnd

m, n, nb = 320, 200, 64
a = rnd(m, n, np.float64, 32)
hist = {}
for tg in ("h", "d"):
    A = s.from_numpy(a, nb=nb, target=tg)
    mt, nt = A.mt, A.nt
    snaps = []
    for k in range(nt):
        cp = A.sub(k, mt - 1, k, k)
        TU = s.geqrf(cp, target=tg)
        snaps.append((f"k{k} geqrf", s.to_numpy(A)))
        if k + 1 < nt:
            A2 = A.sub(k, mt - 1, k + 1, nt - 1)
            s.unmqr(s.Side.Left, s.Op.ConjTrans, cp, TU, A2, target=tg)
            snaps.append((f"k{k} unmqr", s.to_numpy(A)))
            rp = A.sub(k, k, k + 1, nt - 1)
            TV = s.gelqf(rp, target=tg)
            snaps.append((f"k{k} gelqf", s.to_numpy(A)))
            if k + 1 < mt:
                A3 = A.sub(k + 1, mt - 1, k + 1, nt - 1)
                s.unmlq(s.Side.Right, s.Op.ConjTrans, rp, TV, A3, target=tg)
                snaps.append((f"k{k} unmlq", s.to_numpy(A)))
    hist[tg] = snaps
for (name, h), (_, d) in zip(hist["h"], hist["d"]):
    diff = np.abs(h - d)
    idx = np.unravel_index(np.argmax(diff), diff.shape)
    print(f"{name:12s} maxdiff {diff.max():.3e} at {idx}", flush=True)
