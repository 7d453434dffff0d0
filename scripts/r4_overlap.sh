#!/bin/bash
# Stage-2 / stage-1-factor overlap A/B (SLATE_EIG_OVERLAP): GPU eigen tests,
# heev / svd n = 8192.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_overlap; mkdir -p $O
K="heev or svd or bdsqr or hegv or eig" bash scripts/r4_gpu_quick.sh || exit 1
for V in 1 0; do
  SLATE_EIG_OVERLAP=$V EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_o$V.log 2>&1 || { tail $O/heev_o$V.log; exit 1; }
  echo "== overlap=$V"; grep -v "^W20\|amdgpu.ids" $O/heev_o$V.log | head -14
  SLATE_EIG_OVERLAP=$V EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_o$V.log 2>&1 || { tail $O/svd_o$V.log; exit 1; }
  grep -v "^W20\|amdgpu.ids" $O/svd_o$V.log | head -16
done
