#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/qrs
for kc in ${KCS:-8192 16384 4096}; do
  O=gpurun_out/qrs/kc$kc.log
  SLATE_QR_KCHUNK=$kc timeout -k 10 200 python3 bench.py --routines dgeqrf --extras none --check ${CHECK:-no} --steps 1 --warmup 1 > $O 2>&1 || exit $?
  echo "kch=$kc: $(grep -h 'timed\|backward' $O | sed 's/# //' | tr '\n' ' ')"
done
