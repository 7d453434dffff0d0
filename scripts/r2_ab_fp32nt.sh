#!/bin/bash
# A/B: NT vs NN trailing-update form for the fp32 LU inside dgesv_mixed (SLATE_UPDATE_NT), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abf32
for v in 1 0 1b 0b; do
  SLATE_UPDATE_NT=${v:0:1} timeout -k 10 200 python bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none --check yes > gpurun_out/abf32/n$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/abf32/n$v.log; exit 1; }
  echo "nt=$v: $(grep -h -e 'timed' -e iters -e backward gpurun_out/abf32/n$v.log | tr '\n' ' ')"
done
