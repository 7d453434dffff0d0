#!/bin/bash
# Round 6: deferred left interchanges in the one-GPU LU tail (SLATE_LU_DEFER_LEFT = D: defer once the
# remaining matrix is <= m / D tall; 0 = off), dgetrf (tntpiv) + dgetrf_ppiv, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_defer; mkdir -p $O
for d in ${DS:-0 4 2 0 4 8}; do
  SLATE_LU_DEFER_LEFT=$d timeout -k 10 300 python3 -u bench.py --routines dgetrf --extras dgetrf_ppiv --extras-steps 1 --extras-warmup 0 --steps 1 --warmup 1 --check yes > $O/d_$d.json 2> $O/d_$d.err || exit 1
  echo "defer=$d: $(grep -E 'timed|backward' $O/d_$d.err | sed 's/# //' | tr '\n' ' ' | cut -c1-330)"
done
