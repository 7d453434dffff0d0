#!/bin/bash
# Round 6: config 5 on one GPU with the fp32 512-thread tournament trees (SLATE_TSLU_NT=512) vs the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_f32_nt_1gpu; mkdir -p $O
i=0
for rep in 1 2; do
  for nt in 256 512; do
    i=$((i+1))
    SLATE_TSLU_NT=$nt timeout -k 10 300 python3 -u bench.py --routines none --extras cfg5_dgesv_mixed --extras-steps 1 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "nt=$nt: $(grep -E 'phase ms|timed|backward' $O/r$i.err | tail -3 | tr '\n' ' ' | cut -c1-300)"
  done
done
