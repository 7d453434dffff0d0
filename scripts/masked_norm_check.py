import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import slate_d35_amd as s
tg = sys.argv[1]
a = s.utils.random_matrix(700, 700, seed=4)
for up, f in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
    H = s.HermitianMatrix(up, s.from_numpy(a.copy(), nb=128, target=tg))
    h = f(a) + f(a, -1).T if up == s.Uplo.Lower else f(a) + f(a, 1).T
    for k, npk in ((s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro"), (s.Norm.Max, None)):
        ref = np.abs(h).max() if npk is None else np.linalg.norm(h, npk)
        v = s.norm(k, H, target=tg); assert abs(v - ref) < 1e-12 * ref, (up, k, v, ref)
    T = s.TriangularMatrix(up, s.Diag.Unit, s.from_numpy(a.copy(), nb=128, target=tg))
    t = f(a, -1 if up == s.Uplo.Lower else 1) + np.eye(700)
    for k, npk in ((s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro")):
        ref = np.linalg.norm(t, npk); v = s.norm(k, T, target=tg); assert abs(v - ref) < 1e-12 * ref, (up, k, v, ref)
print("masked norms ok", tg)
