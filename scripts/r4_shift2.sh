#!/bin/bash
# bdsqr multishift rounds with 2 / 3 shifts vs the single shift (svd n = 8192).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_shift2; mkdir -p $O
for S in 1 2 3 1 2; do
  SLATE_BDSQR_SHIFTS=$S EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/s$S.log 2>&1 || { tail $O/s$S.log; exit 1; }
  echo "== shifts=$S"; grep -E "^svd| bdsqr |bdsqr_rot_wait" $O/s$S.log
done
