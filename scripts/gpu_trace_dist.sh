#!/bin/bash
# p > 1 lookahead evidence: 2x1 and 2x2 RCCL runs (ranks share the GPU), device-span traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/trace_dist
for g in "2 2 1" "4 2 2"; do
  set -- $g
  timeout -k 10 400 python scripts/rccl_multi.py $1 --cmd python bench.py --gpus $1 --p $2 --q $3 --dim 12288 --nb 512 --routines dgetrf,dgeqrf --steps 1 --warmup 1 --extras none --trace gpurun_out/trace_dist/p$2x$3 > gpurun_out/trace_dist/run_$2x$3.log 2>&1 || { tail -30 gpurun_out/trace_dist/run_$2x$3.log; exit 1; }
  grep -E "timed|backward" gpurun_out/trace_dist/run_$2x$3.log | head -8
  for r in dgetrf dgeqrf; do echo "== $2x$3 $r"; python3 scripts/trace_overlap.py gpurun_out/trace_dist/p$2x$3_$r.json; done
done
rm -f gpurun_out/trace_dist/*.svg
