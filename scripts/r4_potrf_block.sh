#!/bin/bash
# One-workgroup diagonal-block Cholesky (SLATE_POTRF_BLOCK) A/B: GPU potrf
# tests, config 2 (n = 32768, nb = 512) and the 64k dpotrf.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_potrf_block; mkdir -p $O
K="potrf or posv or chol" bash scripts/r4_gpu_quick.sh || exit 1
for cfg in "0 0" "1 0" "1 512" "0 0" "1 0" "1 512"; do
  set -- $cfg
  SLATE_POTRF_BLOCK=$1 SLATE_POTRF_REC_MAX=$2 timeout -k 10 300 python3 bench.py --routines dpotrf --dim 32768 --nb-per dpotrf=512 --steps 3 --warmup 1 --extras none > $O/cfg2_b$1_r$2.log 2>&1 || { tail $O/cfg2_b$1_r$2.log; exit 1; }
  echo "cfg2 block=$1 rec=$2: $(grep -E 'timed|backward' $O/cfg2_b$1_r$2.log | tr '\n' ' ' | cut -c1-260)"
done
for cfg in "0 0" "1 512"; do
  set -- $cfg
  SLATE_POTRF_BLOCK=$1 SLATE_POTRF_REC_MAX=$2 timeout -k 10 300 python3 bench.py --routines dpotrf --steps 2 --warmup 1 --extras none > $O/p64k_b$1_r$2.log 2>&1 || { tail $O/p64k_b$1_r$2.log; exit 1; }
  echo "dpotrf64k block=$1 rec=$2: $(grep -E 'timed|backward' $O/p64k_b$1_r$2.log | tr '\n' ' ' | cut -c1-260)"
done
