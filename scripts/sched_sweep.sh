#!/bin/bash
# panel-starvation knobs on dgetrf / dpotrf at n=65536: K-chunked trailing GEMMs,
# reserved panel CUs, lookahead depth (one process per config)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
for cfg in ${CFGS:-"0 0 1" "512 0 1" "256 0 1" "0 8 1" "0 16 1" "0 0 2" "512 0 2"}; do
  set -- $cfg
  O=gpurun_out/sweep/k$1_c$2_la$3.log
  SLATE_GEMM_KCHUNK=$1 SLATE_PANEL_CUS=$2 timeout -k 10 200 python3 bench.py --routines ${ROUTINES:-dgetrf,dpotrf} --lookahead $3 --extras none --check no --steps 1 --warmup 1 > $O 2>&1 || exit $?
  echo "kchunk=$1 cus=$2 la=$3: $(grep timed $O | sed 's/# //' | tr '\n' ' ')"
done
