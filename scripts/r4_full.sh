#!/bin/bash
# Round 4: full GPU tests, smoke, stage-2 eigen/SVD timings, short headline
# bench.  A plain test failure (pytest exit 1) still lets the later steps run;
# any fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 ${PYTEST_TIMEOUT:-780} python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ -n "${EIG_N:-}" ]; then
  timeout -k 10 300 python -u scripts/eig_prof.py $EIG_N 256 d heev,svd > gpurun_out/eig_prof.log 2>&1 || { tail -20 gpurun_out/eig_prof.log; exit 1; }
  grep -E "^(heev|svd)" gpurun_out/eig_prof.log | head -4
fi
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --extras none ${BENCH_ARGS:-} > gpurun_out/bench_r4.log 2>&1 || { tail -20 gpurun_out/bench_r4.log; exit 1; }
grep -E "timed|backward|metric" gpurun_out/bench_r4.log | tail -3
exit $rc
