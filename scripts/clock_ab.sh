#!/bin/bash
# Effective clock + MFMA busy of our fp64 GEMM vs the vendor yardstick (PMC only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${PMC:-"GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"}
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/clk_ours -o p -- ./tools_bin/gemm_bench_new 8192 > gpurun_out/clk_ours.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/clk_vendor -o p -- python3 scripts/vendor_gemm.py > gpurun_out/clk_vendor.log 2>&1 || exit $?
grep -h "TFLOP" gpurun_out/clk_ours.log gpurun_out/clk_vendor.log
