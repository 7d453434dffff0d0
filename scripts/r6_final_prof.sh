#!/bin/bash
# Round 6 final: kernel trace + stats of the 1-GPU headline suite (bench.py, no extras).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_final_prof; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --extras none --steps 1 --warmup 1 > $O/bench.txt 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.txt | cut -c1-200
db=$(find $O/trace -name "*.db" | head -1)
st=$(find $O/trace -name "*kernel_stats.csv" | head -1)
echo "db=$db stats=$st"
if [ -n "$db" ]; then python3 scripts/prof_summary.py $db 30 > $O/summary.txt; fi
if [ -n "$st" ]; then head -40 $st > $O/kernel_stats_head.csv; fi
ls -la $O $O/trace | head -20
