#!/usr/bin/env python3
"""Timeline analysis of a rocprofv3 kernel trace: how much of the span has a
GEMM running, and what runs when none does.  Usage: timeline.py run_results.db"""
import sqlite3, sys, collections
db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()
gen = [r for r in rows if "generate_kernel" in r[0]]
if gen:  # skip matrix generation
    t_gen_end = max(r[2] for r in gen)
    rows = [r for r in rows if r[1] >= t_gen_end]
t0 = min(r[1] for r in rows); t1 = max(r[2] for r in rows)
def union(iv):
    iv = sorted(iv); out = []
    for s, e in iv:
        if out and s <= out[-1][1]: out[-1][1] = max(out[-1][1], e)
        else: out.append([s, e])
    return out
g = union([(r[1], r[2]) for r in rows if "gemm_mfma" in r[0]])
cov = sum(e - s for s, e in g)
print(f"span {(t1-t0)/1e6:.1f} ms, gemm-covered {cov/1e6:.1f} ms ({100*cov/(t1-t0):.1f}%), gemm-idle {(t1-t0-cov)/1e6:.1f} ms")
# what runs in gemm-idle time
idle = []; prev = t0
for s, e in g:
    if s > prev: idle.append((prev, s))
    prev = max(prev, e)
if t1 > prev: idle.append((prev, t1))
acc = collections.Counter(); anyk = 0
import bisect
for name, s, e, sid in rows:
    if "gemm_mfma" in name: continue
    short = name.split("(")[0].replace("void ", "").replace("slate_amd::dev::", "")[:50]
    for a, b in idle:
        if b <= s: continue
        if a >= e: break
        acc[short] += min(b, e) - max(a, s)
print("non-gemm kernel time inside gemm-idle windows:")
for k, v in acc.most_common(12): print(f"  {v/1e6:9.1f} ms  {k}")
ki = union([(r[1], r[2]) for r in rows])
busy = sum(e - s for s, e in ki)
print(f"GPU fully idle (no kernel at all): {(t1-t0-busy)/1e6:.1f} ms")
# time split in 10 phases
nph = 10
for i in range(nph):
    a = t0 + (t1 - t0) * i / nph; b = t0 + (t1 - t0) * (i + 1) / nph
    c = sum(max(0, min(e, b) - max(s, a)) for s, e in g)
    print(f"  phase {i}: gemm-covered {100*c/(b-a):5.1f}%")
