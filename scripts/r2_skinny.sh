#!/bin/bash
# skinny gemv / trsm kernel tests, then dgesv_mixed at the bench size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "gemv or skinny or gesv_mixed or trsm or gemm" > gpurun_out/skinny_tests.log 2>&1 || { tail -30 gpurun_out/skinny_tests.log; exit 1; }
tail -3 gpurun_out/skinny_tests.log
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --extras none --steps 2 --warmup 1 > gpurun_out/mixed_bench.log 2>&1 || { tail -20 gpurun_out/mixed_bench.log; exit 1; }
grep -h "timed\|phase\|error" gpurun_out/mixed_bench.log
