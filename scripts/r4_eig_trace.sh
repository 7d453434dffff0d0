#!/bin/bash
# Kernel statistics of heev / svd n = 8192 at the end of round 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_eig_trace; mkdir -p $O
for R in heev svd; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$R -o $R -- python3 -u scripts/eig_prof.py 8192 256 d $R > $O/$R.log 2>&1 || { tail $O/$R.log; exit 1; }
  f=$(find $O/$R -name "*kernel_stats.csv" | head -1)
  echo "== $R"; grep -E "^(heev|svd) n=" $O/$R.log; head -14 "$f" | cut -d, -f1-4
done
