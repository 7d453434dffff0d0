#!/bin/bash
# A/B of the bulge chases' sweep grouping (SLATE_SWEEP_GROUP) at n = 8192.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_group; mkdir -p $O
echo "nproc=$(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS"
for G in 1 2 4; do
  SLATE_SWEEP_GROUP=$G EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_g$G.log 2>&1 || { tail $O/heev_g$G.log; exit 1; }
  echo "== G=$G"; grep -E "^heev| hb2st |stedc_dist|residual" $O/heev_g$G.log
  SLATE_SWEEP_GROUP=$G EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd_g$G.log 2>&1 || { tail $O/svd_g$G.log; exit 1; }
  grep -E "^svd| tb2bd | bdsqr " $O/svd_g$G.log
done
