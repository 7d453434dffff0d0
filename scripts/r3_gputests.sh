#!/bin/bash
# full GPU test suite + smoke (as the driver runs them at round end)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/gput; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; exit $rc
