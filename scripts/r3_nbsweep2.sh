#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/nbs2; mkdir -p $O
for cfg in "dgetrf 2048 1" "dgetrf 2048 2" "dgetrf 3072 1" "dgetrf 4096 1" "dpotrf 2048 2" "dgeqrf 1024 2"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --routines $1 --nb $2 --lookahead $3 --steps 1 --warmup 1 --extras none > $O/d.log 2>&1 || { tail -20 $O/d.log; exit 1; }
  echo "== $cfg"; grep -E "timed|backward" $O/d.log | cut -c1-160
done
