#!/bin/bash
# A/B: previous commit (abprev/) vs working tree: dgetrf time; gesv_mixed iterations by tournament form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/abprev; mkdir -p $O
for r in 1 2; do
  for v in abprev .; do
    timeout -k 10 300 python3 $v/bench.py --routines dgetrf --steps 1 --warmup 1 --extras none --check no > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "== $v"; grep -E "timed" $O/b.log
  done
done
for v in "SLATE_TSLU_WG=1" ""; do
  env $v timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none --check no > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 1; }
  echo "== gesv_mixed $v"; grep -E "timed|iters" $O/g.log | cut -c1-160
done
