#!/bin/bash
# A/B: long-K dgemm (n=65536) NN vs TN on a transposed copy of A (SLATE_GEMM_PACK_A), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abpa
for v in 1 0 1b 0b; do
  SLATE_GEMM_PACK_A=${v:0:1} timeout -k 10 200 python bench.py --routines dgemm --steps 2 --warmup 1 --extras none --check yes > gpurun_out/abpa/p$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/abpa/p$v.log; exit 1; }
  echo "packA=$v: $(grep -h -e 'timed' -e backward gpurun_out/abpa/p$v.log | tr '\n' ' ')"
done
