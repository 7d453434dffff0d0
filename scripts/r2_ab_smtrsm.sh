#!/bin/bash
# Batched trtri doubling levels (SLATE_SMALL_TRSM): device kernel tests, then
# config-2 dpotrf (n=32768, nb=512) and n=65536 dpotrf A/B, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/absmtrsm
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_api.py -x -q --timeout 120 -m gpu > gpurun_out/absmtrsm/tests.log 2>&1 || { tail -30 gpurun_out/absmtrsm/tests.log; exit 1; }
tail -1 gpurun_out/absmtrsm/tests.log
for v in 1 0 1b 0b; do
  SLATE_SMALL_TRSM=${v:0:1} timeout -k 10 200 python bench.py --routines dgetrf --steps 1 --warmup 1 --extras cfg5_dgesv_mixed --extras-steps 1 --check yes > gpurun_out/absmtrsm/b$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/absmtrsm/b$v.log; exit 1; }
  echo "batch=$v: $(grep -h -e 'timed' -e backward gpurun_out/absmtrsm/b$v.log | tr '\n' ' ')"
done
