#!/bin/bash
# Sweep-group size 2 vs 3 for the host bulge chases (heev / svd n = 8192).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_group3; mkdir -p $O
for G in 2 3 2 3; do
  SLATE_SWEEP_GROUP=$G EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev,svd > $O/g$G.log 2>&1 || { tail $O/g$G.log; exit 1; }
  echo "== G=$G"; grep -E "^heev|^svd| hb2st | tb2bd " $O/g$G.log
done
