#!/bin/bash
# A/B: getrf trailing update TN (SLATE_UPDATE_TN=1, transposed L21 copy) vs NT, interleaved;
# GPU gemm / getrf tests first (both update forms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abtn
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 -k "gemm or getrf or gesv" > gpurun_out/abtn/tests.log 2>&1 || { tail -30 gpurun_out/abtn/tests.log; exit 1; }
SLATE_UPDATE_TN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 -k "getrf or gesv" > gpurun_out/abtn/tests_tn.log 2>&1 || { tail -30 gpurun_out/abtn/tests_tn.log; exit 1; }
tail -1 gpurun_out/abtn/tests.log; tail -1 gpurun_out/abtn/tests_tn.log
for v in 1 0 1b 0b; do
  SLATE_UPDATE_TN=${v:0:1} timeout -k 10 200 python bench.py --routines dgetrf --steps 2 --warmup 1 --extras none --check yes > gpurun_out/abtn/t$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/abtn/t$v.log; exit 1; }
  echo "tn=$v: $(grep -h -e 'timed' -e backward gpurun_out/abtn/t$v.log | tr '\n' ' ')"
done
