#!/bin/bash
# Round 6: the whole GPU suite verbose (test names as they start), per-test time limits, heartbeat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_suite_v; mkdir -p $O
( while sleep 50; do echo "hb $(date +%T)"; done ) &
hb=$!
timeout -k 10 1300 python3 -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?
kill $hb
grep -E "FAILED|Timeout|passed|failed|ERROR" $O/pytest.txt | head -20
exit $rc
