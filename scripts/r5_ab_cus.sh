#!/bin/bash
# A/B: CUs reserved for the panel / comm queues (SLATE_PANEL_CUS) with the round-5 leaf kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abcus; mkdir -p $O
for v in 0 8 16 0 8; do
  export SLATE_PANEL_CUS=$v
  timeout -k 10 300 python3 -u bench.py --routines dpotrf,dgetrf,dgeqrf --extras cfg2_dpotrf_n32768_nb512 --steps 1 --warmup 1 > $O/c_$v.json 2> $O/c_$v.err || exit 1
  echo "cus=$v: $(grep timed $O/c_$v.err | sed 's/# //; s/ step 1 timed//' | tr '\n' ' ')"
done
