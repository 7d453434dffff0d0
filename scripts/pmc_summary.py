#!/usr/bin/env python3
"""Per-kernel PMC summary from a rocprofv3 --pmc database:
prof db -> for each (kernel, grid) the summed counters.  Usage: pmc_summary.py db [filter]"""
import sqlite3, sys, collections
db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = db.execute("select dispatch_id, kernel_name, grid_size, counter_name, value, duration from counters_collection").fetchall()
agg = collections.OrderedDict()
for did, kn, gs, cn, v, dur in rows:
    if flt and flt not in kn:
        continue
    k = (did, kn[:70], gs)
    d = agg.setdefault(k, {"dur_us": dur / 1e3})
    d[cn] = d.get(cn, 0) + v
for (did, kn, gs), d in agg.items():
    print(f"#{did} {kn} grid={gs} dur={d.pop('dur_us'):.0f}us")
    wc = d.get("SQ_WAVE_CYCLES", 0)
    for cn, v in sorted(d.items()):
        extra = f"  ({100*v/wc:.1f}% of wave cycles)" if wc and cn.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"    {cn:28s} {v:16.0f}{extra}")
