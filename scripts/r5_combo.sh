#!/bin/bash
# probe + focused tests + LU panel composition + dpotrf / dgetrf / dgeqrf / cfg2 / cfg4 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_combo; mkdir -p $O
bash scripts/r5_leafprobe.sh || exit 1
bash scripts/r5_trsm.sh || exit 1
timeout -k 10 600 python3 -u bench.py --routines dpotrf,dgetrf,dgeqrf --extras cfg2_dpotrf_n32768_nb512,cfg4_dgeqrf_nb256 > $O/bench.json 2> $O/bench.err
rc=$?; grep -E "timed" $O/bench.err | tail -12; exit $rc
