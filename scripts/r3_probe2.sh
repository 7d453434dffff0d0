#!/bin/bash
# staircase potrf tests on the multi-rank RCCL rig, then the tail timelines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe2
timeout -k 10 600 python -u -m pytest tests/test_dist.py -x -v --timeout 300 --timeout-method thread -k staircase > gpurun_out/probe2/pytest_stair.log 2>&1 || { tail -40 gpurun_out/probe2/pytest_stair.log; exit 1; }
tail -3 gpurun_out/probe2/pytest_stair.log
bash scripts/r3_tail.sh
