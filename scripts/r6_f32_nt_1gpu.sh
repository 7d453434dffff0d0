#!/bin/bash
# Round 6: config 5 on one GPU: fp32 256-thread tree at <= 256 VGPRs (SLATE_TSLU_F32_WPE=2) vs the default (128, spills).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_f32_nt_1gpu; mkdir -p $O
i=0
for rep in 1 2; do
  for nt in 256 wpe2; do
    i=$((i+1))
    if [ $nt = wpe2 ]; then export SLATE_TSLU_F32_WPE=2; else unset SLATE_TSLU_F32_WPE; fi; timeout -k 10 300 python3 -u bench.py --routines none --extras cfg5_dgesv_mixed --extras-steps 1 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "nt=$nt: $(grep -E 'phase ms|timed|backward' $O/r$i.err | tail -3 | tr '\n' ' ' | cut -c1-300)"
  done
done
