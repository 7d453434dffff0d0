#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cus in ${CUS_LIST:-0 8 32}; do
  SLATE_PANEL_CUS=$cus timeout -k 10 400 python bench.py --routines ${ROUTINES:-dgetrf,dgeqrf} --steps 1 --warmup 0 > gpurun_out/cus_$cus.log 2>&1 || exit $?
  echo "cus=$cus $(grep timed gpurun_out/cus_$cus.log | tr '\n' ' ')"
done
