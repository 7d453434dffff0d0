#!/bin/bash
# Round 6: critical-path model sweep for 2 and 4 GPUs (grid x nb, 32 reserved CUs, CU-free messages).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_sweep24; mkdir -p $O
export SLATE_PANEL_CUS=32
for grid in ${GRIDS:-1x2 2x1 2x2 1x4 4x1}; do
  P=${grid%x*}; Q=${grid#*x}
  for nb in ${NBS:-256 512}; do
    nt=$((65536 / nb)); every=$((nt / 8))
    f=$O/crit_${grid}_nb$nb.txt
    timeout -k 10 300 python3 -u scripts/critpath.py --p $P --q $Q --nb $nb --every $every --reps 2 --routines ${ROUT:-lu,qr,chol} > $f 2>&1 || { tail -5 $f; exit 1; }
    echo "$grid nb=$nb: $(grep -E 'CU-free' $f | sed -E 's/.*-> ([0-9.]+) TFLOP.*/\1/' | tr '\n' ' ')"
  done
done
