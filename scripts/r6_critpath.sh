#!/bin/bash
# Round 6: critical-path model at 2x4 with and without XCD/SE-balanced CU
# reservation for the panel chain (SLATE_PANEL_CUS), messages on the CUs vs
# CU-free (peer copies, host waits inside the chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_crit; mkdir -p $O
for R in ${RS:-0 32}; do
  SLATE_PANEL_CUS=$R timeout -k 10 400 python3 -u scripts/critpath.py --p ${P:-2} --q ${Q:-4} --nb ${NB:-512} --every 16 --reps 2 --routines ${ROUT:-lu,qr,chol} > $O/crit_${P:-2}x${Q:-4}_nb${NB:-512}_R$R.txt 2>&1 || { tail -20 $O/crit_${P:-2}x${Q:-4}_nb${NB:-512}_R$R.txt; exit 1; }
  echo "R=$R"; grep -E "==|steps whose|predicted" $O/crit_${P:-2}x${Q:-4}_nb${NB:-512}_R$R.txt
done
