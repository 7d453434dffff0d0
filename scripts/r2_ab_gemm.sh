#!/bin/bash
# A/B of NN -> NT packing for large products (SLATE_UPDATE_NT) on dgemm n=65536,
# interleaved on one box, then a kernel trace of dgesv_mixed (fp32 LU + fp64
# refinement) at n=65536.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abgemm
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 -k "gemm or trsm or potrf" > gpurun_out/abgemm/tests.log 2>&1 || { tail -20 gpurun_out/abgemm/tests.log; exit 1; }
tail -1 gpurun_out/abgemm/tests.log
for v in 1 0 1b 0b; do
  SLATE_UPDATE_NT=${v:0:1} timeout -k 10 200 python bench.py --routines dgemm --steps 2 --warmup 1 --extras none --check yes > gpurun_out/abgemm/nt$v.log 2>&1 || { echo "nt=$v FAILED"; tail -5 gpurun_out/abgemm/nt$v.log; exit 1; }
  echo "NT=$v: $(grep -h -e 'timed' -e backward gpurun_out/abgemm/nt$v.log | tr '\n' ' ')"
done
R=dgesv_mixed N=65536 BENCH_ARGS="--nb 1024" O=abgemm/prof_mixed bash scripts/prof_qr.sh
