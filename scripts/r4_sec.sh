#!/bin/bash
# Secular-root iteration + host bulge-chase dot/register blocking: GPU eigen
# tests, then heev / svd stage timings at n = 8192.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_sec; mkdir -p $O
K="${K:-stedc or heev or svd or syev or eig}" bash scripts/r4_gpu_quick.sh || exit 1
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev.log 2>&1 || { tail $O/heev.log; exit 1; }
grep -E "^heev|stedc|hb2st|he2hb|residual" $O/heev.log
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd.log 2>&1 || { tail $O/svd.log; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/svd.log | head -30
