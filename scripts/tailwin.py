#!/usr/bin/env python3
"""Panel-stream kernels of one late step: kernel durations and the gaps
between them (launch latency vs execution).  Usage:
    tailwin.py run_results.db [--from-end-ms 60] [--ms 15]"""
import argparse, collections, sqlite3
ap = argparse.ArgumentParser()
ap.add_argument("db"); ap.add_argument("--from-end-ms", type=float, default=60); ap.add_argument("--ms", type=float, default=15)
a = ap.parse_args()
rows = sqlite3.connect(a.db).execute("select name, start, end, stream_id from kernels order by start").fetchall()
t1 = max(r[2] for r in rows)
w0 = t1 - a.from_end_ms * 1e6; w1 = w0 + a.ms * 1e6
win = [r for r in rows if r[1] >= w0 and r[1] < w1]
short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("slate_amd::dev::", "")[:60]
by = collections.defaultdict(list)
for r in win: by[r[3]].append(r)
for sid, rs in by.items():
    busy = sum(r[2] - r[1] for r in rs) / 1e3
    gaps = [(rs[i][1] - rs[i - 1][2]) / 1e3 for i in range(1, len(rs))]
    print(f"stream {sid}: {len(rs)} kernels, busy {busy:.0f} us of {a.ms*1e3:.0f} us, "
          f"mean gap {sum(gaps)/max(1,len(gaps)):.1f} us")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rs:
        k = short(r[0]); agg[k][0] += 1; agg[k][1] += (r[2] - r[1]) / 1e3
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"    {v[0]:5d} x {v[1]/v[0]:8.1f} us  {k}")
    print("  first 60 kernels (start offset us, dur us, gap us):")
    for i, r in enumerate(rs[:60]):
        g = (r[1] - rs[i - 1][2]) / 1e3 if i else 0
        print(f"    {(r[1]-w0)/1e3:9.1f} {(r[2]-r[1])/1e3:8.1f} {g:7.1f}  {short(r[0])}")
