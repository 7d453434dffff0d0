#!/bin/bash
# 1x1 potrf tail (SLATE_POTRF_TAIL: last N columns as one local blocked potrf) after the leaf kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abtail; mkdir -p $O
for t in ${TAILS:-8192 16384 4096 8192 16384}; do
  export SLATE_POTRF_TAIL=$t
  timeout -k 10 200 python3 -u bench.py --routines dpotrf --extras cfg2_dpotrf_n32768_nb512 --steps 1 --warmup 1 > $O/t_$t.json 2> $O/t_$t.err || exit 1
  echo "tail=$t: $(grep -E 'timed' $O/t_$t.err | sed 's/# //; s/ step 1 timed//' | tr '\n' ' ')"
done
