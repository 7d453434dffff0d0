#!/bin/bash
# GPU validation pass: gpu tests, smoke, default bench, device svd/heev tester rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 560 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep -e timed -e metric gpurun_out/bench_default.log
timeout -k 10 300 bin/slate_tester svd,heev --type d,z --dim 2048 --nb 128 --target d > gpurun_out/eig_dev.log 2>&1 || { tail -20 gpurun_out/eig_dev.log; exit 1; }
cat gpurun_out/eig_dev.log
