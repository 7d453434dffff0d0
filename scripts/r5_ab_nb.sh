#!/bin/bash
# nb A/B for dpotrf and dgeqrf after the leaf kernels (1 warm + 1 timed step each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abnb; mkdir -p $O
for nb in 1024 768 1536 1024; do
  timeout -k 10 200 python3 -u bench.py --routines dpotrf --extras none --nb-per dpotrf=$nb --steps 1 --warmup 1 > $O/p_$nb.json 2> $O/p_$nb.err || exit 1
  echo "dpotrf nb=$nb: $(grep timed $O/p_$nb.err | sed 's/# //')"
done
for nb in 512 768 1024 512; do
  timeout -k 10 200 python3 -u bench.py --routines dgeqrf --extras none --nb-per dgeqrf=$nb --steps 1 --warmup 1 > $O/q_$nb.json 2> $O/q_$nb.err || exit 1
  echo "dgeqrf nb=$nb: $(grep timed $O/q_$nb.err | sed 's/# //')"
done
