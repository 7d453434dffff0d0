"""Time the device potrf of one nb x nb diagonal block (the Cholesky / CholeskyQR
panel's latency chain) in isolation: ops.potrf on an SPD matrix, best of reps."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import slate_d35_amd as s
from slate_d35_amd import ops
for nb in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,128,256,512").split(",")]:
    D = torch.rand(nb, nb, dtype=torch.float64, device="cuda")
    D = (D @ D.T + nb * torch.eye(nb, dtype=torch.float64, device="cuda")).contiguous()
    best = 1e9
    for r in range(20):
        X = D.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.potrf("L", X)
        best = min(best, time.perf_counter() - t0)
    L = torch.tril(X.T)   # column-major lower factor
    err = ((L @ L.T) - D).abs().max().item() / D.abs().max().item()
    print(f"potrf nb={nb}: {best*1e6:8.1f} us  err {err:.1e}", flush=True)
