"""Reproduce the wide complex64 device getrf failure after other tests."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
import slate_d35_amd as s
from helpers import rnd, relerr

def run(m, n, dtype, la):
    nb = 128
    a = rnd(m, n, dtype, 21)
    A = s.from_numpy(a, nb=nb, target="d")
    info, piv = s.getrf(A, target="d", lookahead=la)
    f = s.to_numpy(A)
    k = min(m, n)
    L = np.tril(f[:, :k], -1) + np.eye(m, k)
    U = np.triu(f[:k, :])
    ip = [kk * nb + ti * nb + off for kk, pv in enumerate(piv) for (ti, off) in pv]
    pa = a.copy()
    for j, p_ in enumerate(ip):
        pa[[j, p_]] = pa[[p_, j]]
    nanpos = np.argwhere(~np.isfinite(f))
    return info, relerr(L @ U, pa), len(nanpos), nanpos[:3].tolist(), (nanpos[:,0].min(), nanpos[:,0].max(), nanpos[:,1].min(), nanpos[:,1].max()) if len(nanpos) else None

def pre(kind):
    if kind == "singular":
        a = rnd(2000, 64, np.float64, 19); a[:, 5] = 0.0
        tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
        s.ops.getrf_panel(tA, tournament=True)
    elif kind == "tnt":
        for dt in [np.float64, np.complex128, np.float32]:
            for (m, n) in [(1000, 64), (8192, 256), (3000, 100), (70000, 32), (300, 300)]:
                a = rnd(m, n, dt, 18)
                tA = torch.from_numpy(np.ascontiguousarray(a.T)).cuda()
                s.ops.getrf_panel(tA, tournament=True)
    elif kind == "drv":
        for mn in [(700, 700), (900, 500)]:
            for dt in [np.float32, np.float64, np.complex64, np.complex128]:
                run(mn[0], mn[1], dt, 1)
        for dt in [np.float32, np.float64]:
            run(500, 900, dt, 1)
    torch.cuda.synchronize()

for kind in sys.argv[1:]:
    pre(kind)
    for la in [1, 0]:
        r = run(500, 900, np.complex64, la)
        print(kind, "la", la, r, flush=True)
