#!/bin/bash
# permute_rows strips + left swaps off the trailing queue: tests, dgetrf bench, trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/perm; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "getrf or permute or trsm or gesv or lu" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf.log 2>&1 || { tail -20 $O/bench_getrf.log; exit 1; }
grep -E "timed|error" $O/bench_getrf.log
ROUTINES=dgetrf bash scripts/r3_tail.sh > /dev/null 2>&1 || exit 1
head -12 gpurun_out/tail/dgetrf_summary.txt; grep -A12 "gemm-covered" gpurun_out/tail/dgetrf_summary.txt | head -14; tail -1 gpurun_out/tail/dgetrf_steps.txt
