#!/bin/bash
# cfg2 dpotrf (n = 32768, nb = 512): recursive-above-REC_MAX device potrf in
# the 1x1 tail, A/B against the all-blocked sweep, at two tail widths; then
# the 64k dpotrf headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_potrf_rec; mkdir -p $O
K="potrf_kernel or potrf_driver or posv_device" bash scripts/r4_gpu_quick.sh || exit 1
for cfg in "0 8192" "1024 8192" "2048 8192" "1024 12288" "1024 16384"; do
  set -- $cfg
  SLATE_POTRF_REC_MAX=$1 SLATE_POTRF_TAIL=$2 timeout -k 10 300 python3 bench.py --routines dpotrf --dim 32768 --nb-per dpotrf=512 --steps 3 --warmup 1 --extras none > $O/cfg2_r$1_t$2.log 2>&1 || { tail $O/cfg2_r$1_t$2.log; exit 1; }
  echo "cfg2 rec=$1 tail=$2: $(grep -E 'timed|backward' $O/cfg2_r$1_t$2.log | tr '\n' ' ' | cut -c1-300)"
done
for R in 0 1024; do
  SLATE_POTRF_REC_MAX=$R timeout -k 10 300 python3 bench.py --routines dpotrf --steps 2 --warmup 1 --extras none > $O/potrf64k_r$R.log 2>&1 || { tail $O/potrf64k_r$R.log; exit 1; }
  echo "dpotrf64k rec=$R: $(grep -E 'timed|backward' $O/potrf64k_r$R.log | tr '\n' ' ' | cut -c1-300)"
done
