#!/bin/bash
# Round 6: 8-GPU configuration sweep of the critical-path model:
# grid {1x8, 2x4, 4x2} x nb, panel CUs 32 (the multi-process default), for
# LU / QR / Cholesky, plus SUMMA dgemm at K = 512 and 2048 per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_sweep; mkdir -p $O
export SLATE_PANEL_CUS=${R:-32}
for grid in ${GRIDS:-2x4 4x2 1x8}; do
  P=${grid%x*}; Q=${grid#*x}
  for nb in ${NBS:-256 512 1024}; do
    nt=$((65536 / nb)); every=$((nt / 8))
    f=$O/crit_${grid}_nb$nb.txt
    timeout -k 10 300 python3 -u scripts/critpath.py --p $P --q $Q --nb $nb --every $every --reps 2 --routines ${ROUT:-lu,qr,chol} > $f 2>&1 || { tail -5 $f; exit 1; }
    echo "$grid nb=$nb: $(grep -E 'CU-free' $f | sed -E 's/.*-> ([0-9.]+) TFLOP.*/\1/' | tr '\n' ' ')"
  done
done
for grid in 2x4 4x2 1x8; do
  P=${grid%x*}; Q=${grid#*x}
  for K in 512 2048; do
    timeout -k 10 120 python3 -u scripts/critpath.py --p $P --q $Q --nb 512 --summa-k $K --reps 2 --routines gemm 2>&1 | grep "== dgemm" || exit 1
  done
done
