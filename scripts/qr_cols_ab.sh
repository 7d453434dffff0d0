#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SLATE_QR_COLS=1d timeout -k 10 300 python -m pytest tests/test_gpu.py -q -x -k "qr or geqrf or gels or lq" --timeout 120 --timeout-method thread > gpurun_out/qr1d_tests.log 2>&1; rc=$?; tail -2 gpurun_out/qr1d_tests.log; [ $rc -gt 1 ] && exit $rc
for mode in 2d 1d 2d 1d; do
  SLATE_QR_COLS=$mode timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 0 > gpurun_out/qrc_$mode.log 2>&1 || exit $?
  echo "$mode $(grep timed gpurun_out/qrc_$mode.log)"
done
