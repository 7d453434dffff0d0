"""SUMMA-step local GEMM shapes: NT on a copy of B vs TN on a packed A (SLATE_GEMM_PACK_A_MINK)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import slate_d35_amd as s
tag = os.environ.get("SLATE_GEMM_PACK_A_MINK", "2048")
for (m, n, k) in [(32768, 16384, 2048), (16384, 32768, 2048), (32768, 32768, 2048), (32768, 16384, 1024), (65536, 65536, 1024)]:
    a = torch.rand(k, m, dtype=torch.float64, device="cuda")
    b = torch.rand(n, k, dtype=torch.float64, device="cuda")
    c = torch.zeros(n, m, dtype=torch.float64, device="cuda")
    s.ops.gemm("N", "N", 1.0, a, b, 0.0, c); torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps): s.ops.gemm("N", "N", 1.0, a, b, 1.0, c)
    torch.cuda.synchronize(); t = (time.perf_counter() - t0) / reps
    print(f"mink={tag} m={m} n={n} k={k}: {t*1e3:.2f} ms {2*m*n*k/t/1e12:.2f} TF/s", flush=True)
    del a, b, c
    torch.cuda.empty_cache()
