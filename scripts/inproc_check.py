#!/usr/bin/env python3
"""Single process, several in-process ranks (SLATE_INPROC_RANKS, default 4)
through the LAPACK-compatible shim on the device target: dgesv, dgetrf +
dgetrs, dpotrf, dposv, dgemm with residual checks.  On a 1-GPU box all ranks
share device 0 (own contexts / streams each); on an 8-GPU node one per GPU.
Prints INPROC_OK and the per-call wall times."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SLATE_INPROC_RANKS", "4")
os.environ.setdefault("SLATE_LAPACK_NB", "128")
import slate_d35_amd as s  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "slate_d35_amd", "libslate_lapack_api.so"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1536
I = lambda v: C.byref(C.c_int(v))
ptr = lambda a: a.ctypes.data_as(C.c_void_p)
ch = lambda c: C.c_char_p(c.encode())
rel = lambda x, r: np.linalg.norm(x - r) / max(np.linalg.norm(r), 1e-300)
rng = np.random.default_rng(5)
a0 = np.asfortranarray(rng.uniform(-1, 1, (n, n)) + n * np.eye(n))
b0 = np.asfortranarray(rng.uniform(-1, 1, (n, 4)))
info = C.c_int(-1)
ipiv = np.zeros(n, np.int32)
runs0 = s._slate.inproc_run_count()
t = {}

a, b = a0.copy(order="F"), b0.copy(order="F")
t0 = time.time(); L.slate_dgesv_(I(n), I(4), ptr(a), I(n), ptr(ipiv), ptr(b), I(n), C.byref(info)); t["dgesv"] = time.time() - t0
assert info.value == 0 and rel(a0 @ b, b0) < 1e-12, ("gesv", info.value, rel(a0 @ b, b0))
a = a0.copy(order="F")
t0 = time.time(); L.slate_dgetrf_(I(n), I(n), ptr(a), I(n), ptr(ipiv), C.byref(info)); t["dgetrf"] = time.time() - t0
bb = b0.copy(order="F")
L.slate_dgetrs_(ch("N"), I(n), I(4), ptr(a), I(n), ptr(ipiv), ptr(bb), I(n), C.byref(info))
assert rel(a0 @ bb, b0) < 1e-12, ("getrs", rel(a0 @ bb, b0))
h0 = np.asfortranarray(a0 @ a0.T)
h = h0.copy(order="F")
t0 = time.time(); L.slate_dpotrf_(ch("L"), I(n), ptr(h), I(n), C.byref(info)); t["dpotrf"] = time.time() - t0
Lc = np.tril(h)
assert info.value == 0 and rel(Lc @ Lc.T, h0) < 1e-12, ("potrf", info.value)
h, bb = h0.copy(order="F"), b0.copy(order="F")
L.slate_dposv_(ch("U"), I(n), I(4), ptr(h), I(n), ptr(bb), I(n), C.byref(info))
assert info.value == 0 and rel(h0 @ bb, b0) < 1e-9, ("posv", rel(h0 @ bb, b0))
g1, g2 = np.asfortranarray(rng.uniform(-1, 1, (n, n))), np.asfortranarray(rng.uniform(-1, 1, (n, n)))
c = np.zeros((n, n), order="F")
one, zero = C.c_double(1.0), C.c_double(0.0)
t0 = time.time()
L.slate_dgemm_(ch("N"), ch("T"), I(n), I(n), I(n), C.byref(one), ptr(g1), I(n), ptr(g2), I(n), C.byref(zero), ptr(c), I(n))
t["dgemm"] = time.time() - t0
assert rel(c, g1 @ g2.T) < 1e-13, ("gemm", rel(c, g1 @ g2.T))
runs = s._slate.inproc_run_count() - runs0
assert runs == 6, runs
print("INPROC_OK ranks", os.environ["SLATE_INPROC_RANKS"], "grid", s._slate.inproc_last_shape(), "n", n,
      {k: round(v * 1e3, 1) for k, v in t.items()}, "ms", flush=True)
