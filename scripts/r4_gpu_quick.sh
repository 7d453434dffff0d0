#!/bin/bash
# Targeted GPU checks of this round's new device paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_dist.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "${K:-inproc or no_fast_lane or potrf_staircase or native_extension}" > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
