#!/bin/bash
# Eigen / SVD after the local stage 1, one-call back-transforms and the
# one-launch set: GPU eigen tests, heev / svd n = 8192 stage timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_eig_final; mkdir -p $O
K="heev or svd or bdsqr or hegv or eig or set or potrf_driver" bash scripts/r4_gpu_quick.sh || exit 1
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev.log 2>&1 || { tail $O/heev.log; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/heev.log | head -20
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd.log 2>&1 || { tail $O/svd.log; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/svd.log | head -24
