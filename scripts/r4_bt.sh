#!/bin/bash
# One-call stage-1 back-transforms + multishift bdsqr + pipelined rotation
# kernel: GPU eigen tests, heev n = 8192, svd n = 8192 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_bt; mkdir -p $O
K="heev or svd or bdsqr or hegv or eig" bash scripts/r4_gpu_quick.sh || exit 1
SLATE_ROT_PIPE=1 K="bdsqr or svd_device" bash scripts/r4_gpu_quick.sh || exit 1
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev.log 2>&1 || { tail $O/heev.log; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/heev.log | head -16
for cfg in "4 0" "4 1" "1 0" "1 1"; do
  set -- $cfg
  SLATE_BDSQR_SHIFTS=$1 SLATE_ROT_PIPE=$2 EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_s$1_p$2.log 2>&1 || { tail $O/svd_s$1_p$2.log; exit 1; }
  echo "== shifts=$1 pipe=$2"; grep -v "^W20\|amdgpu.ids" $O/svd_s$1_p$2.log | head -12
done
