#!/bin/bash
# Round 6: GEMM-coverage timelines (scripts/coverage.py) of the 1-GPU dgetrf
# (tntpiv, bench defaults), config 2 (dpotrf n=32768 nb=512) and the config-5
# fp32 LU (dgesv_mixed), one timed step each under rocprofv3 --kernel-trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_tl; mkdir -p $O
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- python3 bench.py --steps 1 --warmup 1 --check no "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }
  grep timed $O/$name.log
  CSV=$(find $O/$name -name "*kernel_trace.csv" | head -1)
  python3 scripts/coverage.py $CSV > $O/$name.coverage.txt && cat $O/$name.coverage.txt
  rm -f $CSV
}
run dgetrf --routines dgetrf --extras none && \
run cfg2 --routines none --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 --extras-warmup 1 && \
run fp32lu --routines none --extras cfg5_dgesv_mixed --extras-steps 1 --extras-warmup 1
