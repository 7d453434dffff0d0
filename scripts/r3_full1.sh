#!/bin/bash
# full 1-GPU headline bench (as the driver runs it) + gesv_mixed nb sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/full1; mkdir -p $O
timeout -k 10 700 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -E "timed|error|^\{" $O/bench.log | cut -c1-400
for nb in 512 2048; do
  timeout -k 10 300 python3 bench.py --routines dgesv_mixed --nb $nb --steps 2 --warmup 1 --extras none --check no > $O/g$nb.log 2>&1 || { tail -20 $O/g$nb.log; exit 1; }
  echo "== gesv_mixed nb=$nb"; grep -E "timed|iters" $O/g$nb.log | cut -c1-160
done
