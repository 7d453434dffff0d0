#!/bin/bash
# A/B: lookahead depth for dpotrf / dgeqrf / dgetrf (bench default: 2 / 2 / 1 on one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abla; mkdir -p $O
for la in 0 3 0 3; do
  timeout -k 10 300 python3 -u bench.py --routines dpotrf,dgetrf,dgeqrf --extras cfg2_dpotrf_n32768_nb512,cfg4_dgeqrf_nb256 --lookahead $la --steps 1 --warmup 1 > $O/l_$la.json 2> $O/l_$la.err || exit 1
  echo "la=$la: $(grep timed $O/l_$la.err | sed 's/# //; s/ step 1 timed//' | tr '\n' ' ')"
done
