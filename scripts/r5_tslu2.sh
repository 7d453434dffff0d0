#!/bin/bash
# tournament v2 (256-thread tree): probe, correctness, isolated panel A/B, dgetrf A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_tslu2; mkdir -p $O
for M in 32768 1024; do
  timeout -k 5 60 bin/tslu_probe $M 20 512 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py \
  -k "tournament or getrf or gesv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for MS in "32768 512" "1024 512"; do
  set -- $MS
  PANELS=getrf_tournament timeout -k 10 120 python3 scripts/bench_panel.py $1 $2 2>&1 | grep ms || exit 1
done
timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf.log 2>&1 || { tail $O/bench_getrf.log; exit 1; }
grep -E "dgetrf step|backward" $O/bench_getrf.log
SLATE_TSLU_V1=1 timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf_v1.log 2>&1 || { tail $O/bench_getrf_v1.log; exit 1; }
grep -E "dgetrf step|backward" $O/bench_getrf_v1.log
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 1 --warmup 1 --extras none --check no > $O/bench_mixed.log 2>&1 || { tail $O/bench_mixed.log; exit 1; }
grep -E "step|iters" $O/bench_mixed.log | head -5
SLATE_TSLU_V1=1 timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 1 --warmup 1 --extras none --check no > $O/bench_mixed_v1.log 2>&1 || { tail $O/bench_mixed_v1.log; exit 1; }
grep -E "step|iters" $O/bench_mixed_v1.log | head -5
