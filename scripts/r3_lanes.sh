#!/bin/bash
# Round 3: communication lanes on the multi-rank RCCL rig (ranks share one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lanes
timeout -k 10 900 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/lanes/pytest_dist.log 2>&1 || { tail -40 gpurun_out/lanes/pytest_dist.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/lanes/pytest_dist.log | tail -12
for g in "4 2 2" "8 2 4"; do
  set -- $g
  RANK_TIMEOUT=420 timeout -k 10 450 python scripts/rccl_multi.py $1 --cmd python bench.py --gpus $1 --p $2 --q $3 --dim 8192 --nb 512 --routines dgetrf,dgeqrf --steps 1 --warmup 1 --extras none --trace gpurun_out/lanes/p$2x$3 > gpurun_out/lanes/run_$2x$3.log 2>&1 || { tail -30 gpurun_out/lanes/run_$2x$3.log; exit 1; }
  grep -E "timed|backward" gpurun_out/lanes/run_$2x$3.log | head -8
  for r in dgetrf dgeqrf; do echo "== $2x$3 $r"; python3 scripts/lane_overlap.py gpurun_out/lanes/p$2x$3_$r.json; python3 scripts/trace_overlap.py gpurun_out/lanes/p$2x$3_$r.json | grep -v "top device" ; done
done
rm -f gpurun_out/lanes/*.svg
