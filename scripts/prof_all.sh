#!/bin/bash
# rocprofv3 kernel trace of each headline routine at n=65536 (one run each) + MFMA-busy PMC pass of the dgemm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in dgemm dpotrf dgetrf dgeqrf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pa_$r -o run -- python3 bench.py --routines $r --steps 1 --warmup 0 > gpurun_out/pa_$r.log 2>&1 || exit $?
  grep timed gpurun_out/pa_$r.log
done
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pa_pmc -o p -- python3 bench.py --routines dgemm --steps 1 --warmup 0 > gpurun_out/pa_pmc.log 2>&1 || exit $?
grep timed gpurun_out/pa_pmc.log
