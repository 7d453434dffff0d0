#!/bin/bash
# partial-pivoting dgetrf (the gesv / LAPACK default) tile size A/B, 1 warm + 1 timed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abppiv; mkdir -p $O
for nb in 1024 512 2048 1024; do
  timeout -k 10 200 python3 -u bench.py --routines dgetrf --method-lu ppiv --extras none --nb-per dgetrf=$nb --steps 1 --warmup 1 > $O/p_$nb.json 2> $O/p_$nb.err || exit 1
  echo "ppiv nb=$nb: $(grep -E 'timed|backward' $O/p_$nb.err | sed 's/# //' | tr '\n' ' ')"
done
