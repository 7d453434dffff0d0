#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_bench; mkdir -p $O
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
grep -E "timed|backward|skipped|iters" $O/bench.err | tail -40
tail -1 $O/bench.json | cut -c1-400
exit $rc
