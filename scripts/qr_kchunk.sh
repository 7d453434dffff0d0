#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kc in ${KC_LIST:-0 4096 8192 16384}; do
  SLATE_QR_KCHUNK=$kc timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/qrkc$kc.log 2>&1 || exit $?
  echo "kchunk=$kc $(grep timed gpurun_out/qrkc$kc.log)"
done
