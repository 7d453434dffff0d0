#!/bin/bash
# Round 6: re-decide the panel kernels rejected in round 5 for in-situ slowdowns,
# now under the 32-CU reservation, in the critical-path model at the 8-GPU defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_redecide; mkdir -p $O
export SLATE_PANEL_CUS=32
run() {  # tag env... -- critpath args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u scripts/critpath.py $CP > $O/$tag.txt 2>&1 || { tail -5 $O/$tag.txt; return 1; }
  echo "$tag: $(grep -E 'sampled sums|CU-free messages' $O/$tag.txt | sed -E 's/.*sampled sums: //; s/, contended step.*CU-free comm ([0-9.]+) ms.*/, contended CU-free \1 ms/; s/.*-> ([0-9.]+) TFLOP.*/-> \1/' | tr '\n' ' ')"
}
CP="--p 2 --q 4 --nb 256 --every 32 --reps 2 --routines lu"
run lu_small1 SLATE_SMALL_SOLVE=1 && run lu_small2 SLATE_SMALL_SOLVE=2 && run lu_small1b SLATE_SMALL_SOLVE=1 && run lu_small2b SLATE_SMALL_SOLVE=2 || exit 1
CP="--p 8 --q 1 --nb 512 --every 16 --reps 2 --routines qr"
run qr_sign1 SLATE_LU_SIGN_LEAF=1 && run qr_sign0 SLATE_LU_SIGN_LEAF=0 || exit 1
CP="--p 4 --q 2 --nb 512 --every 16 --reps 2 --routines chol"
run chol_leaf1 SLATE_POTRF_LEAF=1 && run chol_leaf0 SLATE_POTRF_LEAF=0 || exit 1
