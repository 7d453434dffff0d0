#!/bin/bash
# Round 6: the rig's broadcast-mode / no-fast-lane tests with per-test timeouts and a heartbeat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_dist_check; mkdir -p $O
( while sleep 50; do echo "hb $(date +%T)"; done ) &
hb=$!
timeout -k 10 1000 python3 -u -m pytest -v --durations=0 --timeout 240 --timeout-method thread tests/test_dist.py -m gpu -k "bcast_modes or no_fast or staircase" > $O/pytest.txt 2>&1
rc=$?
kill $hb
grep -E "PASSED|FAILED|Timeout|passed|failed|s call" $O/pytest.txt | head -40
exit $rc
