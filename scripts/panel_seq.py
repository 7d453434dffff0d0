#!/usr/bin/env python3
"""Kernel sequence of the LAST repetition of each panel in a bench_panel.py
trace: per-kernel-name count / total / mean, the panel's span and the sum of
inter-kernel gaps (launch latency)."""
import collections, sqlite3, sys
rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("slate_amd::dev::", "")[:70]
# repetitions are separated by a host sync gap > 200 us following a clone (copyBuffer / elementwise)
groups, cur = [], []
for r in rows:
    if cur and r[1] - cur[-1][2] > 200e3:
        groups.append(cur); cur = []
    cur.append(r)
if cur: groups.append(cur)
groups = [g for g in groups if len(g) > 5]
for gi, g in enumerate(groups[-3:]):
    span = (g[-1][2] - g[0][1]) / 1e3
    busy = sum(r[2] - r[1] for r in g) / 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in g:
        k = short(r[0]); agg[k][0] += 1; agg[k][1] += (r[2] - r[1]) / 1e3
    print(f"== group {gi}: {len(g)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {span - busy:.1f} us")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"  {v[0]:5d} x {v[1]/v[0]:8.1f} us = {v[1]:9.1f} us  {k}")
if "--list" in sys.argv and groups:
    # the last repetition kernel by kernel: start offset, duration, gap before it
    g = groups[-1]
    print(f"\n== last group, in order (t0 = first kernel start)")
    prev = g[0][1]
    for r in g:
        print(f"  {(r[1] - g[0][1]) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:8.1f} gap {(r[1] - prev) / 1e3:6.1f}  {short(r[0])}")
        prev = r[2]
