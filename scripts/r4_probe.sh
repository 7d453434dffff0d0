#!/bin/bash
# GEMM probe + svd stage breakdown with the product trace block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_probe; mkdir -p $O
timeout -k 10 120 python3 -u scripts/gemm_probe.py > $O/gemm.log 2>&1 || { tail $O/gemm.log; exit 1; }
grep gemm $O/gemm.log
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd.log 2>&1 || { tail $O/svd.log; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/svd.log | head -24
