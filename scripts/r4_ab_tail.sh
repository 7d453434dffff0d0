#!/bin/bash
# A/B of the potrf tail finish (SLATE_POTRF_TAIL) on config 2 and the headline potrf,
# plus the GPU tests of this round's new paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_ab; mkdir -p $O
for T in 0 4096 8192; do
  SLATE_POTRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dpotrf --dim 32768 --nb-per dpotrf=512 --steps 3 --warmup 1 --extras none > $O/cfg2_tail$T.log 2>&1 || { tail $O/cfg2_tail$T.log; exit 1; }
  echo "cfg2 tail=$T: $(grep -E 'timed|backward' $O/cfg2_tail$T.log | tr '\n' ' ' | cut -c1-400)"
done
for T in 0 4096 8192; do
  SLATE_POTRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dpotrf --steps 2 --warmup 1 --extras none > $O/potrf_tail$T.log 2>&1 || { tail $O/potrf_tail$T.log; exit 1; }
  echo "potrf64k tail=$T: $(grep -E 'timed|backward' $O/potrf_tail$T.log | tr '\n' ' ' | cut -c1-400)"
done
K="inproc or upper or right" bash scripts/r4_gpu_quick.sh
