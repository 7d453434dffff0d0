#!/bin/bash
# Round 3: full GPU tests + smoke + short headline bench (no extras)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --extras none ${BENCH_ARGS:-} > gpurun_out/bench_r3.log 2>&1 || { tail -20 gpurun_out/bench_r3.log; exit 1; }
grep -E "timed|backward" gpurun_out/bench_r3.log
