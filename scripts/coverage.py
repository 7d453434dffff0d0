#!/usr/bin/env python3
"""GEMM-coverage timeline of a factorization from a rocprofv3 kernel trace
(--kernel-trace --output-format csv, or the default .db).

Prints: span, GEMM-covered time (union of every gemm_mfma kernel), per-decile
coverage of the span (decile = tenth of the factorization's wall time), the
GEMM-idle ms per decile, what runs in the idle windows, and the last N
trailing-update steps (the trailing GEMMs on the stream of the longest GEMM:
duration and the idle gap before each).  Matrix generation is skipped.

usage: coverage.py TRACE [--last 10] [--min-us 100]"""
import argparse
import collections
import csv
import os
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=10)
ap.add_argument("--min-us", type=float, default=100.0)
a = ap.parse_args()


def load(path):
    if path.endswith(".csv"):
        out = []
        for r in csv.DictReader(open(path)):
            out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]))
        return sorted(out, key=lambda r: r[1])
    db = sqlite3.connect(path)
    return db.execute("select name, start, end, stream_id from kernels order by start").fetchall()


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("slate_amd::dev::", "")
    return n.split("(")[0][:56]


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


rows = load(a.trace)
gen = [r for r in rows if "generate_kernel" in r[0]]
if gen:
    tg = max(r[2] for r in gen)
    rows = [r for r in rows if r[1] >= tg]
t0, t1 = min(r[1] for r in rows), max(r[2] for r in rows)
span = t1 - t0
g = union([(r[1], r[2]) for r in rows if "gemm_mfma" in r[0] or "gemm_tri" in r[0]])
cov = sum(e - s for s, e in g)
print(f"{os.path.basename(a.trace)}: span {span / 1e6:.1f} ms, gemm-covered {cov / 1e6:.1f} ms "
      f"({100 * cov / span:.1f}%), gemm-idle {(span - cov) / 1e6:.1f} ms")
print(" decile  covered%  idle_ms")
for d in range(10):
    a0, a1 = t0 + span * d / 10, t0 + span * (d + 1) / 10
    c = sum(max(0, min(e, a1) - max(s, a0)) for s, e in g)
    print(f"   {d + 1:2d}     {100 * c / (a1 - a0):6.1f}  {(a1 - a0 - c) / 1e6:7.1f}")
# what runs while no GEMM does
idle, prev = [], t0
for s, e in g:
    if s > prev:
        idle.append((prev, s))
    prev = max(prev, e)
if t1 > prev:
    idle.append((prev, t1))
acc = collections.Counter()
for name, s, e, _ in rows:
    if "gemm_mfma" in name:
        continue
    for x, y in idle:
        if y <= s:
            continue
        if x >= e:
            break
        acc[short(name)] += min(y, e) - max(x, s)
print("non-GEMM kernel time inside GEMM-idle windows:")
for k, v in acc.most_common(8):
    print(f"  {v / 1e6:9.2f} ms  {k}")
busy = sum(e - s for s, e in union([(r[1], r[2]) for r in rows]))
print(f"GPU without any kernel: {(span - busy) / 1e6:.1f} ms")
# last trailing-update steps
big = max((r for r in rows if "gemm_mfma" in r[0]), key=lambda r: r[2] - r[1])
trail = [r for r in rows if r[3] == big[3] and "gemm_mfma" in r[0] and (r[2] - r[1]) >= a.min_us * 1e3]
print(f"last {a.last} trailing GEMMs (stream {big[3]}): start_ms dur_ms gap_before_ms")
for i in range(max(1, len(trail) - a.last), len(trail)):
    r, p = trail[i], trail[i - 1]
    print(f"  {(r[1] - t0) / 1e6:9.2f} {(r[2] - r[1]) / 1e6:7.3f} {(r[1] - p[2]) / 1e6:7.3f}")
