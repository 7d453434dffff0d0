#!/bin/bash
# Round 3: per-step trailing-GEMM / panel timeline of dgetrf and dgeqrf at n=65536
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tail; mkdir -p $O
for R in ${ROUTINES:-dgetrf dgeqrf}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$R -o run -- python3 bench.py --routines $R --steps 1 --warmup 0 --extras none --check no ${BENCH_ARGS:-} > $O/$R.log 2>&1 || { tail -20 $O/$R.log; exit 1; }
  grep timed $O/$R.log
  DB=$(find $O/$R -name "*.db" | head -1)
  python3 scripts/prof_summary.py $DB 25 > $O/${R}_summary.txt && python3 scripts/timeline.py $DB >> $O/${R}_summary.txt
  python3 scripts/steps.py $DB --last 30 > $O/${R}_steps.txt
  python3 scripts/tailwin.py $DB --from-end-ms ${WIN_END:-60} --ms 15 > $O/${R}_win.txt
  cat $O/${R}_summary.txt $O/${R}_steps.txt
  rm -f $DB
done
