#!/usr/bin/env python3
"""How far is tournament pivoting (CALU) from partial pivoting on random
matrices?  Partial pivoting gives |L(i,j)| <= 1 everywhere; a tournament
factorization whose L obeys that bound pivoted exactly as partial pivoting
would have (ties aside): every non-winner row's eliminated entry was at most
the winner's.  So the fraction of panels with max |L| <= 1 is the hit rate of
a tournament-seeded exact PPLU.

usage: l_growth.py [n ...] (defaults 8192 32768); nb = the bench's 2048."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import slate_d35_amd as s  # noqa: E402

ns = [int(x) for x in sys.argv[1:]] or [8192, 32768]
for n in ns:
    for nb in (2048, 512):
        A = s.Matrix(n, n, nb, np.float64)
        A.insertLocalTiles(s.Target.Devices)
        s._slate.generate_matrix_d("rands", A, 7, -1.0, s.opts("d"))
        t0 = time.perf_counter()
        info, piv = s.getrf_tntpiv(A, target="d")
        s.sync()
        dt = time.perf_counter() - t0
        L = s.local_tensor(A)       # n x n, element [i, j] = A(i, j) (column-major strides)
        a = torch.tril(L, -1).abs()
        colmax = a.max(dim=0).values                        # per column max |L|
        tw = 32                                             # tournament block width
        blk = colmax[: n // tw * tw].view(-1, tw).max(dim=1).values
        pan = colmax[: n // nb * nb].view(-1, nb).max(dim=1).values
        print(f"n={n} nb={nb} ({dt * 1e3:.0f} ms): max|L| {a.max().item():.4f}; columns with max|L| > 1: "
              f"{int((colmax > 1).sum())} of {n}; 32-col blocks > 1: {int((blk > 1).sum())} of {blk.numel()}; "
              f"panels > 1: {int((pan > 1).sum())} of {pan.numel()}; entries > 1: {int((a > 1).sum())}",
              flush=True)
        del A, L, a
        torch.cuda.empty_cache()
