"""Compare host vs device results of the ge2tb building blocks on sub-views."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch  # noqa
import slate_d35_amd as s
from helpers import rnd

m, n, nb = 320, 200, 64
a = rnd(m, n, np.float64, 32)
res = {}
for tg in ("h", "d"):
    out = {}
    A = s.from_numpy(a, nb=nb, target=tg)
    rp = A.sub(0, 0, 1, 3)
    Ah = s.from_numpy(np.zeros((rp.n, rp.m)), nb=nb, target=tg)
    s.copy(s.conj_transpose(rp), Ah, target=tg)
    out["copyT"] = s.to_numpy(Ah)
    A = s.from_numpy(a, nb=nb, target=tg)
    rp = A.sub(0, 0, 1, 3)
    T = s.gelqf(rp, target=tg)
    out["gelqf"] = s.to_numpy(A)
    C = s.from_numpy(a[64:, 64:].copy(), nb=nb, target=tg)
    s.unmlq(s.Side.Right, s.Op.ConjTrans, rp, T, C, target=tg)
    out["unmlq"] = s.to_numpy(C)
    A = s.from_numpy(a, nb=nb, target=tg)
    cp = A.sub(0, 4, 0, 0)
    T = s.geqrf(cp, target=tg)
    out["geqrf"] = s.to_numpy(A)
    C = A.sub(0, 4, 1, 3)
    s.unmqr(s.Side.Left, s.Op.ConjTrans, cp, T, C, target=tg)
    out["unmqr"] = s.to_numpy(A)
    res[tg] = out
for k in res["h"]:
    d = np.abs(res["h"][k] - res["d"][k]).max()
    print(f"{k:8s} max|host-device| = {d:.3e}", flush=True)

W = {}
for tg in ("h", "d"):
    A = s.from_numpy(a, nb=nb, target=tg)
    s.ge2tb(A, target=tg)
    W[tg] = s.to_numpy(A)
    print(tg, "band part diff vs host:", np.abs(np.triu(np.tril(W[tg], nb)) - np.triu(np.tril(W["h"], nb))).max(), flush=True)
    sv = np.linalg.svd(np.triu(np.tril(W[tg], nb))[:n], compute_uv=False)
    print(tg, "band svd err", np.abs(sv - np.linalg.svd(a, compute_uv=False)).max(), flush=True)
    A = s.from_numpy(a, nb=nb, target=tg)
    print(tg, "svd_vals err", np.abs(s.svd_vals(A, target=tg) - np.linalg.svd(a, compute_uv=False)).max(), flush=True)
