#!/bin/bash
# WAR fix for the LU left swaps: gesv_mixed determinism + dgetrf timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fix; mkdir -p $O
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none > $O/gesv_mixed.log 2>&1 || { tail -20 $O/gesv_mixed.log; exit 1; }
grep -E "timed|iters|error" $O/gesv_mixed.log | cut -c1-200
for v in "" "SLATE_LU_LEFT_TRAIL=1"; do
  env $v timeout -k 10 300 python3 bench.py --routines dgetrf --steps 2 --warmup 1 --extras none > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  echo "== $v"; grep -E "timed|error" $O/bench.log | cut -c1-200
done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "getrf or gesv or lu" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
