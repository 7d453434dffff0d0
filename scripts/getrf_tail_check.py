import os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import slate_d35_amd as s
rng = np.random.default_rng(3)
for n, nb, meth in [(3000, 256, "tntpiv"), (2500, 512, "partialpiv"), (1000, 128, "tntpiv")]:
    for dt in (np.float64, np.float32, np.complex128):
        a = rng.standard_normal((n, n)).astype(dt)
        if np.iscomplexobj(a): a = a + 1j * rng.standard_normal((n, n))
        b = rng.standard_normal((n, 3)).astype(dt)
        A = s.from_numpy(a, nb=nb, target="d"); B = s.from_numpy(b, nb=nb, target="d")
        info, piv = s.gesv(A, B, target="d", method_lu=meth)
        x = s.to_numpy(B)
        r = np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x) * n * np.finfo(dt).eps)
        print(n, nb, meth, dt.__name__, info, f"{r:.3f}", flush=True)
        assert info == 0 and r < 10, r
print("ok")
