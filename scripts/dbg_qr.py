"""Debug: device geqrf vs numpy for a few shapes/tile sizes (R and Q^H A)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import slate_d35_amd as s

def rnd(m, n, seed):
    return np.random.default_rng(seed).standard_normal((m, n))

for (m, n, nb) in [(260, 260, 64), (300, 64, 64), (260, 64, 64), (1000, 64, 64), (520, 130, 64)]:
    a = rnd(m, n, 3)
    for tg in ("d", "h"):
        A = s.from_numpy(a, nb=nb, target=tg)
        T = s.geqrf(A, target=tg)
        f = s.to_numpy(A)
        k = min(m, n)
        R = np.triu(f[:k])
        C = s.from_numpy(a, nb=nb, target=tg)
        s.unmqr(s.Side.Left, s.Op.ConjTrans, A, T, C, target=tg)
        qa = s.to_numpy(C)
        Rl = np.linalg.qr(a, mode="r")[:k]
        print(m, n, nb, tg, "R vs lapack %.2e" % (np.abs(R - Rl).max() / np.abs(Rl).max()),
              "QhA-R %.2e" % (np.abs(np.triu(qa[:k]) - R).max() / np.abs(R).max()),
              "below %.2e" % (np.abs(qa[k:]).max() if m > k else 0.0), flush=True)
