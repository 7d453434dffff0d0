#!/bin/bash
# Round 6: one-GPU dgetrf: deferred left interchanges from the start (D = 1) and
# the recursive tail (SLATE_GETRF_TAIL) against the default (D = 2, no tail).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_lu_tail; mkdir -p $O
i=0
for rep in 1 2; do
  for cfg in "2 0" "1 0" "2 4096" "2 8192" "1 8192"; do
    set -- $cfg; i=$((i+1))
    SLATE_LU_DEFER_LEFT=$1 SLATE_GETRF_TAIL=$2 timeout -k 10 200 python3 -u bench.py --routines dgetrf --extras none --steps 1 --warmup 1 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "D=$1 tail=$2: $(grep -E 'timed|backward' $O/r$i.err | tr '\n' ' ')"
  done
done
