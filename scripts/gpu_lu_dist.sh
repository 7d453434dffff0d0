#!/bin/bash
# GPU check of the distributed LU: device dist tests (host transport), RCCL
# multi-rank LU on one GPU, the 1-GPU kernel tests, and a 1-GPU dgetrf bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/lu_dist_tests.log 2>&1 || { tail -40 gpurun_out/lu_dist_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/lu_dist_tests.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --routines dgetrf,dgeqrf --steps 1 --warmup 1 > gpurun_out/bench_lu.log 2>&1 || { tail -20 gpurun_out/bench_lu.log; exit 1; }
grep timed gpurun_out/bench_lu.log
