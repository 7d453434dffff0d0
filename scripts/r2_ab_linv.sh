#!/bin/bash
# Once-per-step L(k,k)^{-1} in getrf (SLATE_GETRF_LINV): device LU tests (1x1 and
# a 1x2 grid sharing the GPU), then dgetrf n=65536 + dgesv_mixed A/B, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ablinv
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 -k "getrf or gesv or lu" > gpurun_out/ablinv/tests.log 2>&1 || { tail -30 gpurun_out/ablinv/tests.log; exit 1; }
tail -1 gpurun_out/ablinv/tests.log
timeout -k 10 300 python -u -m pytest tests/test_dist.py -x -q --timeout 280 -m gpu -k "device_shared and 1-2" > gpurun_out/ablinv/dist.log 2>&1 || { tail -30 gpurun_out/ablinv/dist.log; exit 1; }
tail -1 gpurun_out/ablinv/dist.log
for v in 1 0 1b 0b; do
  SLATE_GETRF_LINV=${v:0:1} timeout -k 10 200 python bench.py --routines dgetrf --steps 2 --warmup 1 --extras cfg5_dgesv_mixed --extras-steps 1 --check yes > gpurun_out/ablinv/b$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/ablinv/b$v.log; exit 1; }
  echo "linv=$v: $(grep -h -e 'timed' -e backward gpurun_out/ablinv/b$v.log | tr '\n' ' ')"
done
