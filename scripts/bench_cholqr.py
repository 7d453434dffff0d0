#!/usr/bin/env python3
"""Isolated pieces of one CholeskyQR pass on an mr x nb panel (qr.cc
TsqrPanel::cholqr): G = Q^H Q (herk, lower), L = chol(G) (potrf), Q := Q L^{-H}
(trsm right, lower, conj-trans).  Prints the best of 5 per piece."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import slate_d35_amd as s
from slate_d35_amd import ops

def timed(fn, setup=None, reps=5):
    best = 1e9
    for _ in range(reps):
        args = setup() if setup else ()
        torch.cuda.synchronize(); s.sync()
        t0 = time.perf_counter(); fn(*args); s.sync(); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3

nb = int(os.environ.get("NB", "512"))
for mr in [int(x) for x in (sys.argv[1:] or ["32768", "4096"])]:
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = (torch.rand(nb, mr, dtype=torch.float64, device="cuda", generator=g) * 2 - 1).contiguous()
    G = torch.zeros(nb, nb, dtype=torch.float64, device="cuda")
    t_herk = timed(lambda: ops.herk("L", "C", 1.0, Q, 0.0, G))
    G0 = G.clone()
    t_potrf = timed(lambda X: ops.potrf("L", X), lambda: (G0.clone(),))
    L = G0.clone(); ops.potrf("L", L)
    t_trsm = timed(lambda X: ops.trsm("R", "L", "C", "N", 1.0, L, X), lambda: (Q.clone(),))
    Linv = torch.linalg.inv(torch.tril(L.T)).T.contiguous()   # column-major lower inverse
    W = torch.empty_like(Q)
    t_gemm = timed(lambda: ops.gemm("N", "C", 1.0, Q, Linv, 0.0, W))
    print(f"mr={mr} nb={nb}: herk {t_herk:.3f} potrf {t_potrf:.3f} trsm {t_trsm:.3f} (gemm by L^-H {t_gemm:.3f}) ms", flush=True)
