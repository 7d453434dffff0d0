#!/bin/bash
# lookahead sweep after the round-2 panel changes (one process per setting)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/la3
for cfg in "dgetrf 1" "dgetrf 2" "dpotrf 2" "dpotrf 3" "dgeqrf 2" "dgeqrf 3"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --routines $1 --lookahead $2 --steps 2 --warmup 1 --extras none --check no > gpurun_out/la3/$1_$2.log 2>&1 || { echo "$1 la=$2 FAILED"; tail -5 gpurun_out/la3/$1_$2.log; exit 1; }
  echo "$1 la=$2: $(grep -h 'timed' gpurun_out/la3/$1_$2.log | tr '\n' ' ')"
done
