#!/bin/bash
# Round 6: dgetrf with partial pivoting (the default LU) -- tournament-seeded exact PPLU on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_ppiv; mkdir -p $O
for cfg in ${CFGS:-1:1024 0:1024 1:2048 0:2048 1:1024}; do
  sd=${cfg%%:*}; nb=${cfg##*:}
  SLATE_PPLU_SEED=$sd timeout -k 10 300 python3 -u bench.py --routines none --extras dgetrf_ppiv --extras-steps 1 --extras-warmup 1 --nb-per dgetrf_ppiv=$nb --check yes > $O/c_${sd}_$nb.json 2> $O/c_${sd}_$nb.err || exit 1
  echo "seed=$sd nb=$nb: $(grep -E 'timed|backward' $O/c_${sd}_$nb.err | tr '\n' ' ' | cut -c1-200)"
done
