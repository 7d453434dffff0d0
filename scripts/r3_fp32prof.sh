#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fp32; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 bench.py --routines dgesv_mixed --steps 1 --warmup 0 --extras none --check no > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep -E "timed|iters" $O/b.log | cut -c1-200
DB=$(find $O/tr -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 30 > $O/summary.txt; python3 scripts/timeline.py $DB >> $O/summary.txt; cat $O/summary.txt
python3 scripts/steps.py $DB --last 24 --min-us 100 > $O/steps.txt; cat $O/steps.txt
rm -f $DB
