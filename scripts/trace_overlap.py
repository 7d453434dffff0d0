#!/usr/bin/env python3
"""Lookahead overlap from a --trace JSON (Chrome trace written by
slate::trace::Trace::finish): per rank, how much of the panel work on the
panel queue (tid 101) runs while a trailing-update task is active on the
trailing queue (tid 100).  Usage: trace_overlap.py trace.json [panel_prefix]"""
import json
import sys
from collections import defaultdict

ev = json.load(open(sys.argv[1]))["traceEvents"]
by = defaultdict(lambda: defaultdict(list))
for e in ev:
    if e.get("ph") != "X":
        continue
    by[e["pid"]][e["tid"]].append((e["ts"], e["ts"] + e["dur"], e["name"]))


def union(iv):
    out = []
    for s, t in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], t)
        else:
            out.append([s, t])
    return out


def inter(a, b):
    i = j = 0
    tot = 0.0
    while i < len(a) and j < len(b):
        s, t = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if t > s:
            tot += t - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


for pid in sorted(by):
    lanes = by[pid]
    panel = union([(s, t) for (s, t, n) in lanes.get(101, [])])
    trail = union([(s, t) for (s, t, n) in lanes.get(100, [])])
    comm = union([(s, t) for (s, t, n) in lanes.get(103, [])])
    pt = sum(t - s for s, t in panel)
    tt = sum(t - s for s, t in trail)
    names = defaultdict(float)
    for q in (100, 101, 102, 103):
        for (s, t, n) in lanes.get(q, []):
            names[(q, n)] += t - s
    print(f"rank {pid}: panel-queue busy {pt/1e3:.2f} ms, trailing-queue busy {tt/1e3:.2f} ms, "
          f"panel overlapped by trailing update {inter(panel, trail)/1e3:.2f} ms "
          f"({100*inter(panel, trail)/max(pt,1e-9):.0f}%), comm-queue busy {sum(t-s for s,t in comm)/1e3:.2f} ms, "
          f"comm overlapped by trailing update {inter(comm, trail)/1e3:.2f} ms")
    top = sorted(names.items(), key=lambda kv: -kv[1])[:8]
    print("   top device tasks: " + ", ".join(f"q{q-100}:{n} {v/1e3:.1f}ms" for (q, n), v in top))
