#!/bin/bash
# LU trailing range split over two queues (SLATE_LU_TRAIL_SPLIT): GPU LU
# tests, then dgetrf 64k and dgesv_mixed (fp32 factor) A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_lu_split; mkdir -p $O
K="getrf or gesv or lu_" bash scripts/r4_gpu_quick.sh || exit 1
for S in 0 8 4 16; do
  SLATE_LU_TRAIL_SPLIT=$S timeout -k 10 300 python3 bench.py --routines dgetrf --steps 2 --warmup 1 --extras none > $O/dgetrf_s$S.log 2>&1 || { tail $O/dgetrf_s$S.log; exit 1; }
  echo "dgetrf split=$S: $(grep -E 'timed|backward' $O/dgetrf_s$S.log | tr '\n' ' ' | cut -c1-300)"
done
for S in 0 8; do
  SLATE_LU_TRAIL_SPLIT=$S timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none > $O/mixed_s$S.log 2>&1 || { tail $O/mixed_s$S.log; exit 1; }
  echo "dgesv_mixed split=$S: $(grep -E 'phase|timed|backward' $O/mixed_s$S.log | tr '\n' ' ' | cut -c1-500)"
done
