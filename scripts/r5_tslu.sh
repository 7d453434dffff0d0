#!/bin/bash
# Round 5: tournament v2 correctness + isolated panel A/B (v1 vs v2) + kernel trace + dgetrf.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_tslu; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py \
  -k "tournament or getrf or gesv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for MS in "32768 512" "1024 512" "65536 512"; do
  set -- $MS
  SLATE_TSLU_V1=1 PANELS=getrf_tournament timeout -k 10 120 python3 scripts/bench_panel.py $1 $2 > $O/v1_$1.log 2>&1 || { tail $O/v1_$1.log; exit 1; }
  PANELS=getrf_tournament timeout -k 10 120 python3 scripts/bench_panel.py $1 $2 > $O/v2_$1.log 2>&1 || { tail $O/v2_$1.log; exit 1; }
  echo "v1 $(cat $O/v1_$1.log)"; echo "v2 $(cat $O/v2_$1.log)"
done
PANELS=getrf_tournament timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/bench_panel.py 32768 512 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/panel_kernel_stats.csv \;
head -12 $O/panel_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf.log 2>&1 || { tail $O/bench_getrf.log; exit 1; }
grep -E "dgetrf step|backward" $O/bench_getrf.log
SLATE_TSLU_V1=1 timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench_getrf_v1.log 2>&1 || { tail $O/bench_getrf_v1.log; exit 1; }
grep -E "dgetrf step|backward" $O/bench_getrf_v1.log
