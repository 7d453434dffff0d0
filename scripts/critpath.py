#!/usr/bin/env python3
"""Critical-path harness for the p x q factorizations on ONE GPU.

For a p x q run (default the 8-GPU headline geometry: 2 x 4, n = 65536,
nb = 512) this enqueues, at the real per-process sizes of step k, the tasks
that form the chain from panel k to panel k+1 (getrf.cc getrf_dist /
qr.cc geqrf_impl / potrf.cc), each timed in isolation on the device, and the
trailing update the chain has to hide behind:

  LU (tournament):  local tournament panel (mr x nb, its copy), tree merge
                    (2 nb x nb LU per level), L21 trsm, lookahead column
                    (U solve + GEMM); messages: winners / LU11, L panel
                    (mr x nb) along the row, lookahead row exchange
  QR (TSQR):        local panel QR (mr x nb), tree node QR (2 nb x nb per
                    level), lookahead update (W = V^H C, C -= V T W);
                    messages: (V, T) along the row, W all-reduce down the column
  Cholesky:         diagonal potrf (nb), panel trsm (mr x nb); messages:
                    L panel along the row + transposed tiles over the column

Collectives are not run (one GPU): their time is modelled as
latency + bytes / bandwidth (--lat-us, --bw-gbs: an xGMI ring's per-link
rate) and printed separately.  The isolated task times are a LOWER bound on
the in-run chain (there the panel kernels share CUs with the trailing GEMM).
Output: per sampled step the chain (compute + modelled comm) next to the
per-process trailing update, and the fraction of steps whose chain fits.
"""
import argparse
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import slate_d35_amd as s  # noqa: E402
from slate_d35_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--nb", type=int, default=512)
ap.add_argument("--p", type=int, default=2)
ap.add_argument("--q", type=int, default=4)
ap.add_argument("--la", type=int, default=1)
ap.add_argument("--every", type=int, default=8, help="sample every k-th step")
ap.add_argument("--bw-gbs", type=float, default=64.0, help="modelled per-message bandwidth (GB/s)")
ap.add_argument("--lat-us", type=float, default=25.0, help="modelled per-message latency (us)")
ap.add_argument("--routines", default="lu,qr,chol")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

dev = "cuda"
n, nb, p, q = a.n, a.nb, a.p, a.q
nt = n // nb
g = torch.Generator(device=dev).manual_seed(0)


def rnd(rows, cols):
    # column-major rows x cols == row-major cols x rows
    return (torch.rand(cols, rows, dtype=torch.float64, device=dev, generator=g) * 2 - 1).contiguous()


def timed(fn, setup=None):
    best = math.inf
    for _ in range(a.reps):
        args = setup() if setup else ()
        torch.cuda.synchronize()
        s.sync()
        t0 = time.perf_counter()
        fn(*args)
        s.sync()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3   # ms


def comm(bytes_, msgs=1):
    return msgs * a.lat_us * 1e-3 + bytes_ / (a.bw_gbs * 1e9) * 1e3   # ms


def gemm_ms(m, nn, k, ta="N"):
    if m <= 0 or nn <= 0 or k <= 0:
        return 0.0
    A = rnd(k, m) if ta == "T" else rnd(m, k)
    B = rnd(k, nn)
    C = rnd(m, nn)
    return timed(lambda: ops.gemm(ta, "N", 1.0, A, B, 1.0, C))


def tri(m):
    t = rnd(m, m)
    t += 4 * m * torch.eye(m, dtype=torch.float64, device=dev)   # (symmetric part irrelevant: trsm reads one triangle)
    return t


def rows_local(k):
    """my panel rows at step k (diagonal process: the most)"""
    M = n - k * nb
    return int(math.ceil(M / nb / p)) * nb if M > 0 else 0


def cols_local_trailing(k):
    rest = nt - (k + 1 + a.la)
    return max(0, int(math.ceil(rest / q)) * nb)


def report(name, rows):
    fits = sum(1 for r in rows if r["chain"] <= r["update"])
    print(f"\n== {name}: n={n} nb={nb} grid {p}x{q} la={a.la}; comm model {a.lat_us:.0f} us + bytes/{a.bw_gbs:.0f} GB/s")
    hdr = "   k     mr  nc_trail | " + " ".join(f"{c:>9s}" for c in rows[0]["parts"]) + " |  comm_ms  chain_ms update_ms  fits"
    print(hdr)
    for r in rows:
        parts = " ".join(f"{v:9.3f}" for v in r["parts"].values())
        print(f"{r['k']:4d} {r['mr']:6d} {r['nc']:8d} | {parts} | {r['comm']:8.3f} {r['chain']:9.3f} {r['update']:9.3f}  "
              f"{'yes' if r['chain'] <= r['update'] else 'NO'}")
    tot_chain = sum(r["chain"] for r in rows)
    tot_upd = sum(r["update"] for r in rows)
    print(f"   steps whose chain <= update: {fits}/{len(rows)} ({100.0 * fits / len(rows):.0f}%); "
          f"sampled sums: chain {tot_chain:.1f} ms, update {tot_upd:.1f} ms")
    sys.stdout.flush()


steps = list(range(0, nt - 1, a.every))
todo = a.routines.split(",")

if "lu" in todo:
    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        parts = {}
        W = rnd(mr, nb)
        parts["copy"] = timed(lambda: W.clone())
        parts["tnt_local"] = timed(lambda X: ops.getrf_panel(X, tournament=True), lambda: (W.clone(),))
        lv = max(1, math.ceil(math.log2(p))) if p > 1 else 0
        if lv:
            Sm = rnd(2 * nb, nb)
            parts["tnt_merge"] = lv * timed(lambda X: ops.getrf_panel(X, tournament=True), lambda: (Sm.clone(),))
        else:
            parts["tnt_merge"] = 0.0
        U = tri(nb)
        L21 = rnd(max(mr - nb, 1), nb)
        parts["l21_trsm"] = timed(lambda: ops.trsm("R", "U", "N", "N", 1.0, U, L21))
        Bu = rnd(nb, nb)
        parts["la_u"] = timed(lambda: ops.trsm("L", "L", "N", "U", 1.0, U, Bu))
        parts["la_gemm"] = gemm_ms(mr - nb, nb, nb)
        # messages on the chain: candidates up the tree, winners + LU11 down,
        # pivots + LU11 + L panel along the row, lookahead row exchange
        c = 0.0
        if p > 1:
            c += lv * comm(nb * nb * 8 + nb * 8, 2) + comm(nb * nb * 8, 2) + comm(2 * nb * nb * 8)
        if q > 1:
            c += comm(nb * nb * 8 + 6 * nb * 8, 2) + comm(mr * nb * 8)
        upd = gemm_ms(mr - nb, nc, nb) if nc > 0 else 0.0
        chain = sum(parts.values()) + c
        rows.append(dict(k=k, mr=mr, nc=nc, parts=parts, comm=c, chain=chain, update=upd))
        del W, L21
    report("getrf_tntpiv", rows)

if "qr" in todo:
    # CholeskyQR3 + Householder reconstruction panel (qr.cc TsqrPanel::cholqr)
    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        parts = {}
        Q = rnd(mr, nb)
        G = rnd(nb, nb)
        one_pass = timed(lambda: ops.herk("U", "C", 1.0, Q, 0.0, G))
        D = rnd(nb, nb)
        D = (D @ D.T + nb * torch.eye(nb, dtype=torch.float64, device=dev)).contiguous()
        one_pass += timed(lambda X: ops.potrf("U", X), lambda: (D.clone(),))
        U = tri(nb)
        one_pass += timed(lambda: ops.trsm("R", "U", "N", "N", 1.0, U, Q))
        # CholeskyQR2 (the first attempt; shifted CholeskyQR3 only when the
        # Gram check fails)
        parts["cholqr2"] = 2 * one_pass
        # reconstruction: sign-LU of the kb x kb top block + V = -Q21 U'^{-1}
        Dm = rnd(nb, nb) + 4 * torch.eye(nb, dtype=torch.float64, device=dev)
        parts["hr"] = timed(lambda X: ops.lu_sign(X), lambda: (Dm.clone(),)) + \
            timed(lambda: ops.trsm("R", "U", "N", "N", 1.0, U, Q))
        parts["la_vhc"] = gemm_ms(nb, nb, mr, ta="T")
        parts["la_apply"] = gemm_ms(nb, nb, nb) + gemm_ms(mr, nb, nb)
        c = 0.0
        if p > 1:
            c += 2 * comm(nb * nb * 8) + comm(nb * nb * 8) + comm(nb * nb * 8)   # Gram all-reduces, LU + T, W
        if q > 1:
            c += comm(nb * nb * 8) + comm(mr * nb * 8)
        upd = (gemm_ms(nb, nc, mr, ta="T") + gemm_ms(mr, nc, nb)) if nc > 0 else 0.0
        chain = sum(parts.values()) + c
        rows.append(dict(k=k, mr=mr, nc=nc, parts=parts, comm=c, chain=chain, update=upd))
        del Q
    report("geqrf (CholeskyQR2 + reconstruction panel)", rows)
    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        parts = {}
        W = rnd(mr, nb)
        parts["qr_local"] = timed(lambda X: ops.geqrf_panel(X), lambda: (W.clone(),))
        lv = max(1, math.ceil(math.log2(p))) if p > 1 else 0
        if lv:
            Sm = rnd(2 * nb, nb)
            # tree node QR + Householder reconstruction (~ a second nb-wide factorization)
            parts["tsqr_tree_hr"] = lv * timed(lambda X: ops.geqrf_panel(X), lambda: (Sm.clone(),)) + \
                timed(lambda X: ops.getrf_panel(X, tournament=False), lambda: (rnd(nb, nb),))
        else:
            parts["tsqr_tree_hr"] = 0.0
        # lookahead column: W = V^H C (nb x nb, K = mr), W2 = T^H W, C -= V W2
        parts["la_vhc"] = gemm_ms(nb, nb, mr, ta="T")
        parts["la_apply"] = gemm_ms(nb, nb, nb) + gemm_ms(mr, nb, nb)
        c = 0.0
        if p > 1:
            c += lv * comm(nb * nb * 8, 2) + comm(nb * nb * 8) + comm(nb * nb * 8)   # tree, T down, W all-reduce
        if q > 1:
            c += comm(nb * nb * 8) + comm(mr * nb * 8)                               # (T, V) along the row
        upd = (gemm_ms(nb, nc, mr, ta="T") + gemm_ms(mr, nc, nb)) if nc > 0 else 0.0
        chain = sum(parts.values()) + c
        rows.append(dict(k=k, mr=mr, nc=nc, parts=parts, comm=c, chain=chain, update=upd))
        del W
    report("geqrf (TSQR tree panel, the fallback)", rows)

if "chol" in todo:
    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        parts = {}
        D = rnd(nb, nb)
        D = (D @ D.T + nb * torch.eye(nb, dtype=torch.float64, device=dev)).contiguous()
        parts["potrf_diag"] = timed(lambda X: ops.potrf("L", X), lambda: (D.clone(),))
        L = tri(nb)
        P = rnd(max(mr - nb, 1), nb)
        parts["panel_trsm"] = timed(lambda: ops.trsm("R", "L", "C", "N", 1.0, L, P))
        parts["la_gemm"] = gemm_ms(mr - nb, nb, nb)
        c = 0.0
        if p > 1:
            c += comm(nb * nb * 8)                                  # diag tile down the column
        if q > 1:
            c += comm(mr * nb * 8)                                  # L panel along the row
        if p > 1:
            c += comm(p * math.ceil(nc / nb / max(1, p // 1)) * nb * nb * 8 / max(q, 1))   # transposed tiles
        upd = gemm_ms(mr - nb, nc, nb) if nc > 0 else 0.0
        chain = sum(parts.values()) + c
        rows.append(dict(k=k, mr=mr, nc=nc, parts=parts, comm=c, chain=chain, update=upd))
    report("potrf", rows)
