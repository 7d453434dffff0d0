"""Perf yardstick only: vendor (torch -> hipBLASLt/rocBLAS) fp64 GEMM rates
for the shapes our MFMA kernel serves (never used by the framework)."""
import time
import torch

for (m, n, k) in [(8192, 8192, 8192), (8192, 8192, 512), (16384, 16384, 512)]:
    a = torch.rand(m, k, dtype=torch.float64, device="cuda")
    b = torch.rand(k, n, dtype=torch.float64, device="cuda")
    c = torch.rand(m, n, dtype=torch.float64, device="cuda")
    for _ in range(2):
        c.addmm_(a, b)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        c.addmm_(a, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"vendor dgemm m={m} n={n} k={k}: {2*m*n*k/dt/1e12:.2f} TFLOP/s", flush=True)
