"""Debug: first 16 columns of inv(T) via the skinny trsm, fp32 vs fp64."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import slate_d35_amd as s

for dtype in (np.float64, np.float32):
    for (m, uplo, op, diag) in [(1024, "L", "N", "U"), (2500, "L", "N", "U"), (1024, "L", "N", "N"), (1024, "U", "N", "N")]:
        t = (s.utils.random_matrix(m, m, seed=14, dtype=dtype) / np.sqrt(m) * 0.5 + 2 * np.eye(m)).astype(dtype)
        t = np.tril(t) if uplo == "L" else np.triu(t)
        te = t.astype(np.float64)
        if diag == "U":
            np.fill_diagonal(te, 1)
        cols = list(range(8)) + list(range(512, 520))
        b = np.zeros((m, 16), dtype)
        for r, c in enumerate(cols):
            b[c, r] = 1
        tT = torch.from_numpy(np.ascontiguousarray(t.T)).cuda()
        tB = torch.from_numpy(np.ascontiguousarray(b.T)).cuda()
        s.ops.trsm("L", uplo, "N", diag, dtype(1), tT, tB)
        x = tB.cpu().numpy().T.astype(np.float64)
        ref = np.linalg.solve(te, b.astype(np.float64))
        err = np.abs(x - ref)
        bad = np.argwhere(~(err < 1e-3))
        print(dtype.__name__, m, uplo, diag, "maxerr", np.nanmax(err), "nbad", len(bad), "first bad (row, col)", bad[:8].tolist(), flush=True)
