#!/bin/bash
# dpotrf / dgetrf at n=65536: lookahead and panel-CU sweep (one step each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "1 0" "2 0" "3 0" "1 16" "2 16"; do
  set -- $cfg
  SLATE_PANEL_CUS=$2 timeout -k 10 200 python3 bench.py --routines dpotrf,dgetrf --steps 2 --warmup 1 --lookahead $1 --extras none --check no > gpurun_out/la_$1_$2.log 2>&1 || { tail -5 gpurun_out/la_$1_$2.log; exit 1; }
  echo "la=$1 cus=$2: $(grep -o '"routines".*' gpurun_out/la_$1_$2.log | head -c 600)"
done
