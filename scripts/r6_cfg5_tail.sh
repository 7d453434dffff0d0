#!/bin/bash
# Round 6: config-5 fp32 factor with the recursive LU tail (SLATE_GETRF_TAIL) and nb.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_cfg5_tail; mkdir -p $O
i=0
for rep in 1 2; do
  for cfg in "0 1024" "4096 1024" "8192 1024" "0 2048"; do
    set -- $cfg; i=$((i+1))
    SLATE_GETRF_TAIL=$1 timeout -k 10 300 python3 -u bench.py --routines none --extras cfg5_dgesv_mixed --extras-steps 1 --nb-per cfg5_dgesv_mixed=$2 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "tail=$1 nb=$2: $(grep -E 'phase ms|timed' $O/r$i.err | tail -2 | tr '\n' ' ' | cut -c1-260)"
  done
done
