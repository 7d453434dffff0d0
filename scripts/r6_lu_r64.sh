#!/bin/bash
# Round 6: LU critical-path model at 2 x 4 / nb 256 and 1 x 8 / nb 256 with 32 / 64 / 96 reserved CUs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_lu_r64; mkdir -p $O
for g in "2 4" "1 8"; do
  set -- $g
  for R in 32 64 96; do
    SLATE_PANEL_CUS=$R timeout -k 10 300 python3 -u scripts/critpath.py --p $1 --q $2 --nb 256 --every 32 --reps 2 --routines lu > $O/crit_${1}x${2}_R$R.txt 2>&1 || { tail -5 $O/crit_${1}x${2}_R$R.txt; exit 1; }
    echo "${1}x${2} R=$R: $(grep -E 'sampled sums|CU-free messages' $O/crit_${1}x${2}_R$R.txt | sed -E 's/.*sampled sums: //; s/.*-> ([0-9.]+) TFLOP.*/-> \1/' | tr '\n' ' ')"
  done
done
