#!/bin/bash
# wave-per-leaf tournament select: panel tests, isolated panel A/B, dgetrf bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tslu; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "tournament or getrf or trsm" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for mode in 0 1; do
  for m in 2048 8192 32768; do
    SLATE_TSLU_WG=$mode PANELS=tournament timeout -k 10 120 python3 scripts/bench_panel.py $m 1024 2>&1 | grep -v "^W2026\|amdgpu.ids" | sed "s/^/wg=$mode /" >> $O/panel.txt || exit 1
  done
done
cat $O/panel.txt
timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf.log 2>&1 || { tail -20 $O/bench_getrf.log; exit 1; }
grep -E "timed|error" $O/bench_getrf.log
