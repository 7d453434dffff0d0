#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_cq; mkdir -p $O
timeout -k 10 200 python3 -u scripts/bench_cholqr.py 32768 4096 > $O/times.log 2>&1 || { tail $O/times.log; exit 1; }
grep mr= $O/times.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/p -o run -- python3 scripts/bench_cholqr.py 32768 > $O/p.log 2>&1 || { tail $O/p.log; exit 1; }
DB=$(find $O/p -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 30 > $O/summary.txt 2>&1; rm -rf $O/p
head -34 $O/summary.txt
