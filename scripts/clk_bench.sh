#!/bin/bash
# Effective clock / MFMA busy of the bench's dgemm vs the standalone harness at the same size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/clkb_bench -o p -- python3 bench.py --routines dgemm --steps 1 --warmup 0 > gpurun_out/clkb_bench.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/clkb_std -o p -- ./tools_bin/gemm_bench_rot1 65536 65536 0 1 > gpurun_out/clkb_std.log 2>&1 || exit $?
grep -h "TFLOP" gpurun_out/clkb_bench.log gpurun_out/clkb_std.log
