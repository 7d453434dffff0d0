#!/usr/bin/env python3
"""Critical-path harness for the p x q factorizations on ONE GPU.

For a p x q run (default the 8-GPU headline geometry: 2 x 4, n = 65536,
nb = 512) this enqueues, at the real per-process sizes of step k, the tasks
that form the chain from panel k to panel k+1 (getrf.cc getrf_dist /
qr.cc geqrf_impl / potrf.cc) and the trailing update the chain has to hide
behind:

  LU (tournament):  local tournament panel (mr x nb, its copy), tree merge
                    (2 nb x nb LU per level), L21 trsm, lookahead column
                    (U solve + GEMM), the host wait for the pivot slots
                    (getrf.cc); messages: winners / LU11, L panel (mr x nb)
                    along the row, lookahead row exchange
  QR (CholeskyQR2): two Gram (herk) + potrf + trsm passes, the host check of
                    the Gram matrix (qr.cc), Householder reconstruction,
                    lookahead update; messages: Gram all-reduces, (V, T)
                    along the row, W all-reduce; the TSQR tree (the fallback)
                    is reported too
  Cholesky:         diagonal potrf (nb), panel trsm (mr x nb), lookahead GEMM;
                    messages: L panel along the row + transposed tiles; the
                    update is the lower-trapezoid part each process owns (the
                    staircase launch), not its full local rectangle
  dgemm:            SUMMA: one local (n/p x n/q x nb) GEMM per step against
                    the two panel messages

Per sampled step three times are measured:
  chain   the chain's tasks one after another, alone on the GPU (+ the
          modelled messages: latency + bytes / bandwidth, --lat-us / --bw-gbs;
          collectives are not run, there is one GPU)
  update  the step's trailing update alone
  step    the chain's tasks on the high-priority panel queue WHILE the
          trailing update GEMM runs on the trailing queue -- the lookahead-1
          schedule of the drivers, with its CU contention -- plus the
          modelled messages
The prediction is sum_k step_k (sampled steps scaled by --every) and the
whole-node TFLOP/s it implies (LAWN-41 flops).  Run at 1 x 1 it predicts the
one-GPU drivers, which checks the model against the driver-timed numbers.
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
ap.add_argument("--routines", default="lu,qr,chol,gemm")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--summa-k", type=int, default=2048, help="SUMMA K per step (gemmC: w = K / nb tiles per step)")
a = ap.parse_args()

dev = "cuda"
n, nb, p, q = a.n, a.nb, a.p, a.q
nt = n // nb
g = torch.Generator(device=dev).manual_seed(0)
ops.set_queue(1)   # chain tasks on the panel queue, as in the drivers
# torch's own work (operand copies) on a non-blocking stream: with CU-masked
# queues (SLATE_PANEL_CUS, created blocking) any legacy-null-stream op would
# be a device-wide barrier between the chain and the update
torch.cuda.set_stream(torch.cuda.Stream())


def rnd(rows, cols):
    # column-major rows x cols == row-major cols x rows
    return (torch.rand(cols, rows, dtype=torch.float64, device=dev, generator=g) * 2 - 1).contiguous()


def sync_all():
    s.sync()
    torch.cuda.synchronize()


def comm(bytes_, msgs=1):
    return msgs * a.lat_us * 1e-3 + bytes_ / (a.bw_gbs * 1e9) * 1e3   # ms


def tri(m):
    t = rnd(m, m)
    t += 4 * m * torch.eye(m, dtype=torch.float64, device=dev)   # (trsm reads one triangle)
    return t


def spd(m):
    D = rnd(m, m)
    return (D @ D.T + m * torch.eye(m, dtype=torch.float64, device=dev)).contiguous()


class Task:
    """One chain task: fn(*setup()) on the panel queue (the binding waits for it)."""

    def __init__(self, name, fn, setup=None):
        self.name, self.fn, self.setup = name, fn, setup or (lambda: ())


class Gemm:
    """A GEMM (m x nn x k, op(A) = A or A^T) launched on a queue without waiting."""

    def __init__(self, m, nn, k, ta="N"):
        self.ok = m > 0 and nn > 0 and k > 0
        if self.ok:
            self.A = rnd(k, m) if ta == "T" else rnd(m, k)
            self.B, self.C, self.ta = rnd(k, nn), rnd(m, nn), ta

    def launch(self, queue):
        if self.ok:
            ops.gemm_async(queue, self.ta, "N", 1.0, self.A, self.B, 1.0, self.C)


def measure(tasks, updates, cm):
    """(per-task alone, chain alone, update alone, contended step, contended
    step with CU-free comm), ms, best of reps.

    step    = the chain's kernels on the panel queue while the update runs,
              plus the modelled messages added on top (messages on the CUs,
              serialized with the chain: RCCL kernels);
    step_ov = the same with the messages as host waits INSIDE the chain,
              right before its lookahead task (a copy-engine transport,
              SLATE_BCAST=peer: the bytes move while the update runs)."""
    alone = {}
    for t in tasks:
        best = math.inf
        for _ in range(a.reps):
            args = t.setup()
            sync_all()
            t0 = time.perf_counter()
            t.fn(*args)
            best = min(best, time.perf_counter() - t0)
        alone[t.name] = best * 1e3
    upd = math.inf
    for _ in range(a.reps):
        sync_all()
        t0 = time.perf_counter()
        for u in updates:
            u.launch(0)
        ops.queue_sync(0)
        upd = min(upd, time.perf_counter() - t0)
    step = math.inf
    for _ in range(a.reps):
        args = [t.setup() for t in tasks]
        sync_all()
        t0 = time.perf_counter()
        for u in updates:
            u.launch(0)
        for t, ar in zip(tasks, args):
            t.fn(*ar)
        ops.queue_sync(0)
        step = min(step, time.perf_counter() - t0)
    step_ov = math.inf
    # the messages land before the lookahead task (the last GEMM-like task)
    la_at = min([i for i, t in enumerate(tasks) if t.name.startswith("la_")] or [len(tasks)])
    for _ in range(a.reps):
        args = [t.setup() for t in tasks]
        sync_all()
        t0 = time.perf_counter()
        for u in updates:
            u.launch(0)
        for i, (t, ar) in enumerate(zip(tasks, args)):
            if i == la_at and cm > 0:
                t1 = time.perf_counter()
                while time.perf_counter() - t1 < cm * 1e-3:
                    pass
            t.fn(*ar)
        if la_at >= len(tasks) and cm > 0:
            t1 = time.perf_counter()
            while time.perf_counter() - t1 < cm * 1e-3:
                pass
        ops.queue_sync(0)
        step_ov = min(step_ov, time.perf_counter() - t0)
    return alone, sum(alone.values()) + cm, upd * 1e3, step * 1e3 + cm, step_ov * 1e3


def host_wait_task():
    X = rnd(8, 8) + 8 * torch.eye(8, dtype=torch.float64, device=dev)
    return Task("host_wait", lambda Y: ops.potrf("L", Y), lambda: (X.clone(),))


def rows_local(k):
    """my panel rows at step k (diagonal process: the most)"""
    M = n - k * nb
    return int(math.ceil(M / nb / p)) * nb if M > 0 else 0


def cols_local_trailing(k):
    rest = nt - (k + 1 + a.la)
    return max(0, int(math.ceil(rest / q)) * nb)


def lawn41(name):
    if name.startswith("getrf"):
        return 2.0 / 3.0 * n ** 3
    if name.startswith("geqrf"):
        return 4.0 / 3.0 * n ** 3
    return n ** 3 / 3.0


def report(name, rows):
    print(f"\n== {name}: n={n} nb={nb} grid {p}x{q} la={a.la}; comm model {a.lat_us:.0f} us + bytes/{a.bw_gbs:.0f} GB/s")
    hdr = "   k     mr  nc_trail | " + " ".join(f"{c:>9s}" for c in rows[0]["parts"]) + \
        " |  comm_ms  chain_ms update_ms   step_ms  fits"
    print(hdr + "   step_ov")
    for r in rows:
        parts = " ".join(f"{v:9.3f}" for v in r["parts"].values())
        print(f"{r['k']:4d} {r['mr']:6d} {r['nc']:8d} | {parts} | {r['comm']:8.3f} {r['chain']:9.3f} "
              f"{r['update']:9.3f} {r['step']:9.3f}  {'yes' if r['chain'] <= r['update'] else 'NO '} "
              f"{r['step_ov']:9.3f}")
    fits = sum(1 for r in rows if r["chain"] <= r["update"])
    tc, tu, ts, to = (sum(r[x] for r in rows) for x in ("chain", "update", "step", "step_ov"))
    tmax = sum(max(r["chain"], r["update"]) for r in rows)
    print(f"   steps whose chain <= update: {fits}/{len(rows)} ({100.0 * fits / len(rows):.0f}%); "
          f"sampled sums: chain {tc:.1f} ms, update {tu:.1f} ms, contended step {ts:.1f} ms, "
          f"with CU-free comm {to:.1f} ms; sum max(chain, update) {tmax:.1f} ms -> "
          f"contended / max = {ts / tmax:.2f} (CU-free comm {to / tmax:.2f})")
    for lab, t in (("messages on the CUs", ts), ("CU-free messages (peer copies)", to)):
        pred = t * a.every
        print(f"   predicted ({lab}): sum_k step x {a.every} = {pred:.0f} ms -> "
              f"{lawn41(name) / (pred * 1e-3) / 1e12:.1f} TFLOP/s whole node ({p}x{q}, panel CUs "
              f"{os.environ.get('SLATE_PANEL_CUS', '0')})")
    sys.stdout.flush()


steps = list(range(0, nt - 1, a.every))
todo = a.routines.split(",")

if "lu" in todo:
    rows = []
    lv = max(1, math.ceil(math.log2(p))) if p > 1 else 0
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        W = rnd(mr, nb)
        Sm = rnd(2 * nb, nb)
        U = tri(nb)
        L21 = rnd(max(mr - nb, 1), nb)
        Bu = rnd(nb, nb)
        la = Gemm(mr - nb, nb, nb)
        tasks = [Task("copy", lambda: W.clone()),
                 Task("tnt_local", lambda X: ops.getrf_panel(X, tournament=True), lambda: (W.clone(),))]
        tasks += [Task(f"merge{i}", lambda X: ops.getrf_panel(X, tournament=True), lambda: (Sm.clone(),))
                  for i in range(lv)]
        tasks += [Task("l21_trsm", lambda: ops.trsm("R", "U", "N", "N", 1.0, U, L21)),
                  Task("la_u", lambda: ops.trsm("L", "L", "N", "U", 1.0, U, Bu)),
                  Task("la_gemm", lambda: (la.launch(1), ops.queue_sync(1))),
                  host_wait_task()]
        c = 0.0
        if p > 1:
            c += lv * comm(nb * nb * 8 + nb * 8, 2) + comm(nb * nb * 8, 2) + comm(2 * nb * nb * 8)
        if q > 1:
            c += comm(nb * nb * 8 + 6 * nb * 8, 2) + comm(mr * nb * 8)
        alone, chain, upd, step, step_ov = measure(tasks, [Gemm(mr - nb, nc, nb)] if nc > 0 else [], c)
        rows.append(dict(k=k, mr=mr, nc=nc, parts=alone, comm=c, chain=chain, update=upd, step=step, step_ov=step_ov))
        del W, L21
    report("getrf_tntpiv", rows)

if "qr" in todo:
    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        Q = rnd(mr, nb)
        G = rnd(nb, nb)
        D = spd(nb)
        U = tri(nb)
        Dm = rnd(nb, nb) + 4 * torch.eye(nb, dtype=torch.float64, device=dev)
        vhc, ap1, ap2 = Gemm(nb, nb, mr, ta="T"), Gemm(nb, nb, nb), Gemm(mr, nb, nb)
        # as the driver (qr.cc cholqr): Lower Gram, Lower Cholesky (the leaf
        # kernel's path), Q L^-H
        one = [Task("gram", lambda: ops.herk("L", "C", 1.0, Q, 0.0, G)),
               Task("potrf", lambda X: ops.potrf("L", X), lambda: (D.clone(),)),
               Task("trsm", lambda: ops.trsm("R", "L", "C", "N", 1.0, U, Q))]
        tasks = [Task(t.name + str(i), t.fn, t.setup) for i in range(2) for t in one]   # CholeskyQR2
        tasks += [host_wait_task(),
                  Task("hr_lu", lambda X: ops.lu_sign(X), lambda: (Dm.clone(),)),
                  Task("hr_trsm", lambda: ops.trsm("R", "U", "N", "N", 1.0, U, Q)),
                  Task("la_update", lambda: (vhc.launch(1), ap1.launch(1), ap2.launch(1), ops.queue_sync(1)))]
        c = 0.0
        if p > 1:
            c += 2 * comm(nb * nb * 8) + comm(nb * nb * 8) + comm(nb * nb * 8)   # Gram all-reduces, LU + T, W
        if q > 1:
            c += comm(nb * nb * 8) + comm(mr * nb * 8)
        upds = [Gemm(nb, nc, mr, ta="T"), Gemm(mr, nc, nb)] if nc > 0 else []
        alone, chain, upd, step, step_ov = measure(tasks, upds, c)
        rows.append(dict(k=k, mr=mr, nc=nc, parts=alone, comm=c, chain=chain, update=upd, step=step, step_ov=step_ov))
        del Q
    report("geqrf (CholeskyQR2 + reconstruction panel)", rows)

if "chol" in todo:
    def stair_fraction(k):
        """Largest per-process share of the lower-trapezoid trailing tiles
        (I >= J) relative to that process's full local rectangle."""
        best = 0.0
        for pr in range(p):
            for pc in range(q):
                rows_ = [I for I in range(k + 1, nt) if I % p == pr]
                cols_ = [J for J in range(k + 1 + a.la, nt) if J % q == pc]
                if rows_ and cols_:
                    own = sum(1 for J in cols_ for I in rows_ if I >= J)
                    best = max(best, own / (len(rows_) * len(cols_)))
        return best

    rows = []
    for k in steps:
        mr, nc = rows_local(k), cols_local_trailing(k)
        D = spd(nb)
        L = tri(nb)
        P = rnd(max(mr - nb, 1), nb)
        la = Gemm(mr - nb, nb, nb)
        tasks = [Task("potrf_diag", lambda X: ops.potrf("L", X), lambda: (D.clone(),)),
                 Task("panel_trsm", lambda: ops.trsm("R", "L", "C", "N", 1.0, L, P)),
                 Task("la_gemm", lambda: (la.launch(1), ops.queue_sync(1)))]
        c = 0.0
        if p > 1:
            c += comm(nb * nb * 8)                                  # diag tile down the column
        if q > 1:
            c += comm(mr * nb * 8)                                  # L panel along the row
        if p > 1:
            c += comm(p * nb * nb * 8)                              # lookahead column's transposed tiles (first all-gather)
        ncs = int(nc * stair_fraction(k)) // nb * nb if nc > 0 else 0
        alone, chain, upd, step, step_ov = measure(tasks, [Gemm(mr - nb, ncs, nb)] if ncs > 0 else [], c)
        rows.append(dict(k=k, mr=mr, nc=nc, parts=alone, comm=c, chain=chain, update=upd, step=step, step_ov=step_ov))
    report("potrf", rows)

if "gemm" in todo:
    # SUMMA: every process multiplies its (n/p x n/q) block, K = nb per step;
    # the panel broadcasts overlap the previous step's GEMM
    mloc, nloc = n // p, n // q
    w = max(1, a.summa_k // nb)
    G1 = Gemm(mloc, nloc, w * nb)
    best = math.inf
    for _ in range(a.reps):
        sync_all()
        t0 = time.perf_counter()
        for _ in range(8):
            G1.launch(0)
        ops.queue_sync(0)
        best = min(best, (time.perf_counter() - t0) / 8)
    per_k = best * 1e3
    c = w * (comm(mloc * nb * 8) + comm(nb * nloc * 8)) if p * q > 1 else 0.0
    steps_ = math.ceil(nt / w)
    pred = steps_ * max(per_k, c)
    print(f"\n== dgemm: n={n} nb={nb} grid {p}x{q} SUMMA K={w * nb} per step: local GEMM {per_k:.3f} ms, "
          f"comm {c:.3f} ms; predicted {pred:.0f} ms -> {2.0 * n ** 3 / (pred * 1e-3) / 1e12:.1f} TFLOP/s whole node")
