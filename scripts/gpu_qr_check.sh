#!/bin/bash
# GPU check of the QR panel: kernel/driver tests, tester residuals (s/d/c/z),
# 1-GPU dgeqrf bench (TSQR narrow panel vs column path A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 bin/slate_tester geqrf,gels,gelqf,heev,svd --type s,d,c,z --dim 1000,2500x700,700x1300 --nb 256 --target d > gpurun_out/qr_tester.log 2>&1 || { tail -30 gpurun_out/qr_tester.log; exit 1; }
tail -3 gpurun_out/qr_tester.log
timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 1 > gpurun_out/bench_qr.log 2>&1 || { tail -20 gpurun_out/bench_qr.log; exit 1; }
grep timed gpurun_out/bench_qr.log
SLATE_QR_PANEL=columns timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 1 > gpurun_out/bench_qr_cols.log 2>&1 || { tail -20 gpurun_out/bench_qr_cols.log; exit 1; }
grep timed gpurun_out/bench_qr_cols.log
