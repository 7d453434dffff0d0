#!/bin/bash
# dgetrf n = 65536 on one GPU: lookahead x nb sweep (same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_lu_sweep; mkdir -p $O
for cfg in "2048 1" "2048 2" "1536 1" "1536 2" "1024 2"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --routines dgetrf --nb-per dgetrf=$1 --lookahead $2 --steps 2 --warmup 1 --extras none > $O/nb$1_la$2.log 2>&1 || { tail $O/nb$1_la$2.log; exit 1; }
  echo "nb=$1 la=$2: $(grep -E 'timed' $O/nb$1_la$2.log | tr '\n' ' ' | cut -c1-200)"
done
