#!/bin/bash
# Local he2hb / ge2tb + one-call stage-1 back-transforms: GPU eigen tests,
# heev / svd n = 8192 stage timings (and the driver-form A/B for he2hb/ge2tb).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_bt; mkdir -p $O
K="heev or svd or bdsqr or hegv or eig" bash scripts/r4_gpu_quick.sh || exit 1
for L in 1 0; do
  SLATE_HE2HB_LOCAL=$L SLATE_GE2TB_LOCAL=$L EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_l$L.log 2>&1 || { tail $O/heev_l$L.log; exit 1; }
  echo "== local=$L"; grep -v "^W20\|amdgpu.ids" $O/heev_l$L.log | head -16
  SLATE_HE2HB_LOCAL=$L SLATE_GE2TB_LOCAL=$L EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_l$L.log 2>&1 || { tail $O/svd_l$L.log; exit 1; }
  grep -v "^W20\|amdgpu.ids" $O/svd_l$L.log | head -16
done
for KD in 32 48; do
  SLATE_EIG_KD=$KD EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_kd$KD.log 2>&1 || { tail $O/heev_kd$KD.log; exit 1; }
  echo "== kd=$KD"; grep -v "^W20\|amdgpu.ids" $O/heev_kd$KD.log | head -8
  SLATE_EIG_KD=$KD EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_kd$KD.log 2>&1 || { tail $O/svd_kd$KD.log; exit 1; }
  grep -v "^W20\|amdgpu.ids" $O/svd_kd$KD.log | head -8
done
