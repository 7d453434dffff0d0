#!/bin/bash
# Trailing-update GEMM shapes (general vs lower-triangle, NT / NN / TN) and a
# kernel trace of dgesv_mixed at the bench size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "32768 1024 3" "16384 1024 5" "32768 512 3" "49152 1024 2"; do
  timeout -k 10 120 ./tools_bin/gemm_bench tri $a >> gpurun_out/tri_sweep.txt 2>&1 || exit $?
done
cat gpurun_out/tri_sweep.txt
O=prof_mixed
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$O -o run -- python3 bench.py --routines dgesv_mixed --extras none --check no --steps 1 --warmup 0 > gpurun_out/$O.log 2>&1 || exit $?
grep -h "timed\|phase" gpurun_out/$O.log
