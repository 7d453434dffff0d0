#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu.py -q -x -k "qr or geqrf or gels or lq or heev or svd or unmqr" --timeout 120 --timeout-method thread > gpurun_out/qr_tests.log 2>&1; rc=$?; tail -2 gpurun_out/qr_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/qrb_$i.log 2>&1 || exit $?
  echo "$(grep timed gpurun_out/qrb_$i.log)"
done
