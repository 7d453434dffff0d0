#!/bin/bash
# Round-3 final: the driver's 1-GPU bench, then per-routine kernel traces with the GEMM timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 700 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -E "timed|error|^\{" $O/bench.log | cut -c1-300
for R in dgetrf dgeqrf dpotrf; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$R -o run -- python3 bench.py --routines $R --steps 1 --warmup 0 --extras none --check no > $O/$R.log 2>&1 || { tail -20 $O/$R.log; exit 1; }
  DB=$(find $O/$R -name "*.db" | head -1)
  { grep timed $O/$R.log; python3 scripts/prof_summary.py $DB 20; python3 scripts/timeline.py $DB; python3 scripts/steps.py $DB --last 12; } > $O/trace_$R.txt
  rm -f $DB
  head -3 $O/trace_$R.txt
done
