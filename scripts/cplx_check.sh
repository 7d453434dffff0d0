#!/bin/bash
# complex MFMA GEMM: kernel/driver tests (s/d/c/z), tester throughput of c/z routines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 bin/slate_tester gemm,herk,potrf,getrf_tntpiv,geqrf,trsm --type c,z --dim 2000 --nb 256 --target d > gpurun_out/cplx_tester.log 2>&1 || { tail -30 gpurun_out/cplx_tester.log; exit 1; }
tail -14 gpurun_out/cplx_tester.log
timeout -k 10 300 bin/slate_tester gemm --type z,c --dim 16384 --nb 512 --target d --check n > gpurun_out/cplx_perf.log 2>&1 || { tail -30 gpurun_out/cplx_perf.log; exit 1; }
timeout -k 10 300 bin/slate_tester potrf,getrf_tntpiv --type z --dim 32768 --nb 512 --target d --check n >> gpurun_out/cplx_perf.log 2>&1 || { tail -30 gpurun_out/cplx_perf.log; exit 1; }
cat gpurun_out/cplx_perf.log
