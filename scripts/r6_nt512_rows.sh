#!/bin/bash
# Round 6: one-GPU dgetrf with 512-thread tournament trees for short panels only (SLATE_TSLU_NT512_ROWS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_nt512_rows; mkdir -p $O
i=0
for rep in 1 2; do
  for t in 0 8192 16384 32768; do
    i=$((i+1))
    SLATE_TSLU_NT512_ROWS=$t timeout -k 10 200 python3 -u bench.py --routines dgetrf --extras none --steps 1 --warmup 1 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "rows<=$t: $(grep -E 'timed|backward' $O/r$i.err | tr '\n' ' ')"
  done
done
