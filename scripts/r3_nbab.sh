#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/nbab; mkdir -p $O
for r in 1 2; do
for cfg in "dgeqrf 512 2" "dgeqrf 1024 2" "dpotrf 1024 2" "dpotrf 2048 2" "dpotrf 2048 1"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --routines $1 --nb $2 --lookahead $3 --steps 1 --warmup 1 --extras none --check no > $O/d.log 2>&1 || { tail -20 $O/d.log; exit 1; }
  echo "== $cfg: $(grep -E 'step 1 timed' $O/d.log)"
done
done
