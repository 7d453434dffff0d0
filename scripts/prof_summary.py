#!/usr/bin/env python3
"""Summarize a rocprofv3 rocpd database: per-kernel total time, count, avg.
Usage: prof_summary.py run_results.db [topN]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = db.execute("select name, start, end from kernels").fetchall()
agg = {}
t0 = min(r[1] for r in rows); t1 = max(r[2] for r in rows)
for name, s, e in rows:
    short = name.replace("void ", "").replace("slate_amd::dev::", "").replace("(anonymous namespace)::", "")
    short = re.sub(r"\(long.*|\(char.*|\(int.*|\(bool.*", "", short)[:100]
    a = agg.setdefault(short, [0, 0])
    a[0] += e - s
    a[1] += 1
tot = sum(v[0] for v in agg.values())
print(f"kernels: {len(rows)} dispatches, kernel-time sum {tot/1e6:.1f} ms, span {(t1-t0)/1e6:.1f} ms")
print(f"{'ms':>10} {'%':>6} {'count':>7} {'avg_us':>9}  kernel")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{v[0]/1e6:10.2f} {100*v[0]/tot:6.1f} {v[1]:7d} {v[0]/v[1]/1e3:9.1f}  {k}")
