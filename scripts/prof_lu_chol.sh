#!/bin/bash
# kernel traces of dgetrf (tntpiv and ppiv) and dpotrf at the bench size + GEMM timelines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_lu
for R in "dgetrf tntpiv" "dpotrf tntpiv" "dgetrf ppiv"; do
  set -- $R
  O=gpurun_out/prof_lu/$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O -o run -- python3 bench.py --routines $1 --method-lu $2 --extras none --check no --steps 1 --warmup 0 > $O.log 2>&1 || exit $?
  grep timed $O.log
  DB=$(find $O -name "*.db" | head -1)
  { grep timed $O.log; python3 scripts/prof_summary.py $DB 14; python3 scripts/timeline.py $DB; } > $O.txt 2>&1
  cat $O.txt
  find $O -name "*.db" -delete
done
