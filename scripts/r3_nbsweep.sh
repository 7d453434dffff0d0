#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/nbs; mkdir -p $O
for nb in 1024 1536 2048; do
  timeout -k 10 300 python3 bench.py --routines dgesv_mixed --nb $nb --steps 2 --warmup 1 --extras none --check no > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 1; }
  echo "== gesv_mixed nb=$nb"; grep -E "timed|iters" $O/g.log | cut -c1-160
done
for nb in 1536 2048; do
  timeout -k 10 300 python3 bench.py --routines dgetrf --nb $nb --steps 1 --warmup 1 --extras none > $O/d.log 2>&1 || { tail -20 $O/d.log; exit 1; }
  echo "== dgetrf nb=$nb"; grep -E "timed|backward" $O/d.log | cut -c1-160
done
