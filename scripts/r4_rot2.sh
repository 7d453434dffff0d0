#!/bin/bash
# bdsqr: pipelined rotation kernel (Hin prefetch, LDS-only barrier) x
# multishift rounds, svd n = 8192 A/B; GPU tests with the pipe kernel first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_rot2; mkdir -p $O
SLATE_ROT_PIPE=1 K="bdsqr or svd_device" bash scripts/r4_gpu_quick.sh || exit 1
for cfg in "1 0" "1 1" "2 1" "3 1" "2 0"; do
  set -- $cfg
  SLATE_BDSQR_SHIFTS=$1 SLATE_ROT_PIPE=$2 EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/s$1_p$2.log 2>&1 || { tail $O/s$1_p$2.log; exit 1; }
  echo "== shifts=$1 pipe=$2"; grep -E "^svd| bdsqr |bdsqr_rot_wait" $O/s$1_p$2.log
done
