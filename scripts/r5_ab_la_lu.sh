#!/bin/bash
# dgetrf lookahead 1 (1-GPU default) vs 2, interleaved, 1 warm + 2 timed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_ablalu; mkdir -p $O
for la in 1 2 1 2; do
  timeout -k 10 200 python3 -u bench.py --routines dgetrf --extras none --lookahead $la --steps 2 --warmup 1 > $O/l_$la.json 2> $O/l_$la.err || exit 1
  echo "dgetrf la=$la: $(grep -E 'timed' $O/l_$la.err | sed 's/# //' | tr '\n' ' ')"
done
