import torch, time, sys
sys.path.insert(0, '/root/repo')
import slate_d35_amd as s
n = 8192
for shape in ("NN",):
    a = torch.rand(n, n, dtype=torch.float64, device="cuda"); b = torch.rand(n, n, dtype=torch.float64, device="cuda"); c = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    s.ops.gemm("N", "N", 1.0, a, b, 0.0, c); torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(3): s.ops.gemm("N", "N", 1.0, a, b, 0.0, c)
    torch.cuda.synchronize(); t = (time.time() - t0) / 3
    print(f"gemm {shape} n={n}: {t*1e3:.1f} ms {2*n**3/t/1e12:.1f} TF/s", flush=True)
