#!/bin/bash
# Kernel trace of one routine at the bench size: prof_routine.sh <routine> [out]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-dgeqrf}; O=${2:-prof_$R}
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/$O -o run -- python3 bench.py --routines $R --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/$O.log 2>&1 || exit $?
grep timed gpurun_out/$O.log
