#!/bin/bash
# GPU validation run: pytest -m gpu, smoke, short bench.  Stops at the first
# crash/timeout (exit > 1); plain test failures (exit 1) continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--n 32768 --steps 2 --warmup 1"}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; cat gpurun_out/smoke.log | tail -5
if [ $rc -ne 0 ]; then echo "smoke rc=$rc -> stop"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; tail -20 gpurun_out/bench.log
exit $rc
