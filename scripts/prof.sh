#!/bin/bash
# rocprofv3 kernel trace + stats of a bench run (args passed to bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 bench.py "$@" > $OUT/bench.log 2>&1
rc=$?
tail -5 $OUT/bench.log
find $OUT -name "*kernel_stats.csv" | head -3 | while read f; do echo "== $f"; head -25 "$f"; done
exit $rc
