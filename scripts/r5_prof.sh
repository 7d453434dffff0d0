#!/bin/bash
# kernel statistics of one step of each suite routine (rocprofv3 --kernel-trace --stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_prof; mkdir -p $O
for R in dgeqrf dpotrf dgemm dgetrf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$R -o run --output-format csv -- python3 bench.py --routines $R --steps 1 --warmup 0 --extras none --check no > $O/$R.log 2>&1 || { tail $O/$R.log; exit 1; }
  f=$(find $O/$R -name "*kernel_stats.csv" | head -1)
  cp $f $O/${R}_kernel_stats.csv
  grep "step 0" $O/$R.log
  head -8 $O/${R}_kernel_stats.csv | cut -d, -f1-5
  find $O/$R -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
