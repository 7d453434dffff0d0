#!/bin/bash
# Wave-pipelined bdsqr rotation kernel: GPU tests, then svd n = 8192 A/B
# (SLATE_ROT_PIPE=0: single-wave kernel) and a kernel-trace of the new one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_rot; mkdir -p $O
K="bdsqr or svd or heev_device" bash scripts/r4_gpu_quick.sh || exit 1
for P in 1 0; do
  SLATE_ROT_PIPE=$P EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_p$P.log 2>&1 || { tail $O/svd_p$P.log; exit 1; }
  echo "== pipe=$P"; grep -E "^svd| tb2bd | bdsqr |bdsqr_rot" $O/svd_p$P.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o svd -- python3 -u scripts/eig_prof.py 8192 256 d svd > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} head -8 {}
