#!/bin/bash
# Sliding-window stage-2 back-transform A/B + heev / svd stage timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_eig2; mkdir -p $O
K="${K:-stage2_fused or heev_device or svd_device}" bash scripts/r4_gpu_quick.sh || exit 1
for S in 1 0; do
  SLATE_HB2ST_SLIDE=$S EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_slide$S.log 2>&1 || { tail $O/heev_slide$S.log; exit 1; }
  echo "== slide=$S"; grep -E "^heev|unmtr_hb2st|hb2st |residual" $O/heev_slide$S.log
done
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd.log 2>&1; grep -v "^W20\|amdgpu.ids" $O/svd.log | head -30
