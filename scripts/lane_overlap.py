#!/usr/bin/env python3
"""Communication-lane evidence from a --trace JSON (device spans per Sched
task, tid 100 + queue): per rank, how many critical-path lane spans on the
panel queue (q1: tournament / panel gather / TSQR / pivot, LU11, L, (V, T)
broadcasts, lookahead exchanges) START while a bulk-lane span on the comm
queue (q3: trailing row exchanges, left swaps, trailing W all-reduces) is
still running -- with one in-order comm queue these would all have waited
for the bulk span to finish.  Usage: lane_overlap.py trace.json"""
import json
import sys
from collections import defaultdict

ev = json.load(open(sys.argv[1]))["traceEvents"]
by = defaultdict(lambda: defaultdict(list))
for e in ev:
    if e.get("ph") == "X":
        by[e["pid"]][e["tid"]].append((e["ts"], e["ts"] + e["dur"], e["name"]))
CRIT = ("getrf_tnt_send", "getrf_tnt_recv", "getrf_bcast_winners", "getrf_panel_perm", "getrf_bcast_row",
        "getrf_bcast_L", "getrf_pp_panel", "getrf_rows_exchange", "geqrf_tsqr_sendR", "geqrf_tsqr_recvR",
        "geqrf_tsqr_recvE", "geqrf_tsqr_sendE", "geqrf_tsqr_bcast_lu", "geqrf_bcast", "geqrf_update_allreduce")
BULK = ("getrf_rows_exchange", "getrf_left_swap", "geqrf_update_allreduce")
for pid in sorted(by):
    q1 = sorted(x for x in by[pid][101] if x[2] in CRIT)
    q3 = sorted(x for x in by[pid][103] if x[2] in BULK)
    early = 0
    for s, t, n in q1:
        if any(bs < s < bt for bs, bt, _ in q3):
            early += 1
    busy3 = sum(t - s for s, t, _ in q3) / 1e3
    busy1 = sum(t - s for s, t, _ in q1) / 1e3
    print(f"rank {pid}: critical-lane spans {len(q1)} ({busy1:.1f} ms), bulk-lane spans {len(q3)} ({busy3:.1f} ms); "
          f"critical spans starting while a bulk span runs: {early}")
