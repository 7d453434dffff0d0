#!/usr/bin/env python3
"""Per-step view of a factorization's kernel trace: for every trailing-update
GEMM (kernels on the stream that runs the longest GEMM), its start, duration,
the idle gap on that stream before it, and how long the panel stream (the
stream of the panel kernels named by --panel) was busy between the previous
trailing GEMM's end and this one's start.  Usage:
    steps.py run_results.db [--panel tslu,qr_node,potrf] [--last N]"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--panel", default="tslu,qr_node,lu_sign,potrf_inv,tsip,qr_hr")
ap.add_argument("--last", type=int, default=40)
ap.add_argument("--min-us", type=float, default=300.0)
a = ap.parse_args()
db = sqlite3.connect(a.db)
rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()
gen = [r for r in rows if "generate_kernel" in r[0]]
if gen:
    tg = max(r[2] for r in gen)
    rows = [r for r in rows if r[1] >= tg]
t0 = rows[0][1]
big = max((r for r in rows if "gemm_mfma" in r[0]), key=lambda r: r[2] - r[1])
trail = big[3]
pkeys = a.panel.split(",")
panel = [r for r in rows if any(k in r[0] for k in pkeys)]
pstream = max(set(r[3] for r in panel), key=lambda s: sum(1 for r in panel if r[3] == s)) if panel else -1
tg_ = [r for r in rows if r[3] == trail and "gemm_mfma" in r[0] and (r[2] - r[1]) / 1e3 >= a.min_us]
ptimes = sorted((r[1], r[2]) for r in rows if r[3] == pstream)
print(f"trail stream {trail}, panel stream {pstream}, {len(tg_)} trailing GEMMs >= {a.min_us} us")
print(f"{'#':>4} {'t_ms':>9} {'gemm_ms':>8} {'gap_ms':>7} {'panel_busy_ms':>13} {'panel_span_ms':>13}")
prev_end = None
out = []
for i, r in enumerate(tg_):
    s, e = r[1], r[2]
    gap = (s - prev_end) / 1e6 if prev_end is not None else 0.0
    w0 = prev_end if prev_end is not None else t0
    # panel work between the previous trailing GEMM's START and this one's start
    ws = tg_[i - 1][1] if i > 0 else t0
    busy = sum(max(0, min(pe, s) - max(ps, ws)) for ps, pe in ptimes) / 1e6
    inwin = [(ps, pe) for ps, pe in ptimes if pe > ws and ps < s]
    span = (max(pe for _, pe in inwin) - min(ps for ps, _ in inwin)) / 1e6 if inwin else 0.0
    out.append((i, (s - t0) / 1e6, (e - s) / 1e6, gap, busy, span))
    prev_end = e
for o in out[-a.last:]:
    print(f"{o[0]:4d} {o[1]:9.1f} {o[2]:8.2f} {o[3]:7.2f} {o[4]:13.2f} {o[5]:13.2f}")
tot_gap = sum(o[3] for o in out)
print(f"total trailing-stream gap between trailing GEMMs: {tot_gap:.1f} ms; "
      f"last-10 steps gap {sum(o[3] for o in out[-10:]):.1f} ms, gemm {sum(o[2] for o in out[-10:]):.1f} ms")
