"""Time the device sign-modified LU (Householder reconstruction step of the
CholeskyQR panel) of one n x n block in isolation, best of reps; checks
L U = A + diag(s)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import slate_d35_amd as s
from slate_d35_amd import ops
for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "256,512,1024").split(",")]:
    torch.manual_seed(0)
    Q, _ = torch.linalg.qr(torch.randn(2 * n, n, dtype=torch.float64, device="cuda"))
    D = (-Q[:n, :n]).T.contiguous()          # column-major -Q11, as the HR step factors
    best = 1e9
    for r in range(10):
        X = D.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sg = ops.lu_sign(X)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    F = X.T
    L = torch.tril(F, -1) + torch.eye(n, dtype=F.dtype, device=F.device)
    U = torch.triu(F)
    S = torch.diag(torch.tensor(sg, dtype=F.dtype, device=F.device))
    err = ((L @ U) - (D.T + S)).abs().max().item()
    print(f"lu_sign n={n}: {best*1e6:8.1f} us  err {err:.1e}", flush=True)
