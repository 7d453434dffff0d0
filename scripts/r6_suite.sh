#!/bin/bash
# Round 6: the whole GPU test suite (one pytest process), summary to gpurun_out/r6_suite/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_suite; mkdir -p $O
timeout -k 10 1300 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?
tail -15 $O/pytest.txt
exit $rc
