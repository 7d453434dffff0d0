#!/usr/bin/env python3
"""Per-kernel durations of the panel chain alone vs while a long trailing GEMM
runs, from a rocprofv3 --kernel-trace CSV (critpath.py under rocprofv3).

usage: contention.py kernel_trace.csv [min_gemm_ms]
A kernel counts as 'contended' when it overlaps a GEMM of >= min_gemm_ms
(default 1) on another queue."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("slate_amd::dev::", "")
    r["name"] = nm.split("(")[0][:48]
big = [r for r in rows if "gemm" in r["name"] and (r["e"] - r["s"]) >= min_ms * 1e6]
stats = defaultdict(lambda: [[], []])
for r in rows:
    if r in big:
        continue
    cont = any(b["Queue_Id"] != r["Queue_Id"] and r["s"] < b["e"] and r["e"] > b["s"] for b in big)
    stats[r["name"]][1 if cont else 0].append((r["e"] - r["s"]) / 1e3)
print(f"{'kernel':48s} {'n_alone':>7s} {'us_alone':>9s} {'n_cont':>7s} {'us_cont':>9s} {'ratio':>6s}")
for name, (a, c) in sorted(stats.items(), key=lambda kv: -sum(kv[1][1])):
    if not c:
        continue
    ma = sorted(a)[len(a) // 2] if a else float("nan")
    mc = sorted(c)[len(c) // 2]
    print(f"{name:48s} {len(a):7d} {ma:9.1f} {len(c):7d} {mc:9.1f} {mc / ma if a else float('nan'):6.2f}")
