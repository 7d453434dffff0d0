#!/bin/bash
# Round 6: tournament step with the row-broadcast wave max and 16-byte row
# publish (SLATE_TSLU_FAST=1, default) vs the round-5 step (=0): isolated
# panels, the 2x4 / nb 256 LU critical-path model, the 1-GPU dgetrf.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_tslu_fast; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "tournament or tntpiv" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for f in 0 1 0 1; do
  for mn in "32768 512" "1024 512" "32768 256" "512 256"; do
    SLATE_TSLU_FAST=$f PANELS=tournament timeout -k 10 120 python3 -u scripts/bench_panel.py $mn 2>&1 | grep getrf | sed "s/^/fast=$f /" | tee -a $O/panels.txt || exit 1
  done
done
for f in 0 1; do
  SLATE_TSLU_FAST=$f SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 2 --q 4 --nb 256 --every 32 --reps 2 --routines lu > $O/crit_fast$f.txt 2>&1 || { tail -5 $O/crit_fast$f.txt; exit 1; }
  echo "fast=$f: $(grep -E 'sampled sums|CU-free messages' $O/crit_fast$f.txt | tr '\n' ' ' | cut -c1-400)"
done
for f in 0 1 0 1; do
  SLATE_TSLU_FAST=$f timeout -k 10 300 python3 -u bench.py --routines dgetrf --extras none --steps 1 --warmup 1 > $O/lu_$f.txt 2> $O/lu_$f.err || { tail -20 $O/lu_$f.err; exit 1; }
  echo "fast=$f: $(grep -E 'timed|backward' $O/lu_$f.err | tr '\n' ' ')"
done
