#!/bin/bash
# Round 6: 512-thread tournament tree workgroups (SLATE_TSLU_NT=512: 1024-row
# leaves, fan-in 32, one level fewer) vs 256: correctness, isolated panels,
# the 2x4 / nb 256 and 1x8 LU models with 32 reserved CUs, the 1-GPU dgetrf.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_tslu_nt; mkdir -p $O
SLATE_TSLU_NT=512 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "tournament or tntpiv" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for nt in 256 512 256 512; do
  for mn in "32768 512" "32768 256" "8192 256" "512 256"; do
    SLATE_TSLU_NT=$nt PANELS=tournament timeout -k 10 120 python3 -u scripts/bench_panel.py $mn 2>&1 | grep getrf | sed "s/^/nt=$nt /" | tee -a $O/panels.txt || exit 1
  done
done
for nt in 256 512 256 512; do
  SLATE_TSLU_NT=$nt SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 2 --q 4 --nb 256 --every 32 --reps 2 --routines lu > $O/crit_$nt.txt 2>&1 || { tail -5 $O/crit_$nt.txt; exit 1; }
  echo "2x4 nt=$nt: $(grep -E 'sampled sums|CU-free messages' $O/crit_$nt.txt | sed -E 's/.*sampled sums: //; s/, contended step.*CU-free comm ([0-9.]+) ms.*/, contended CU-free \1 ms/; s/.*-> ([0-9.]+) TFLOP.*/-> \1/' | tr '\n' ' ')"
done
for nt in 256 512; do
  SLATE_TSLU_NT=$nt timeout -k 10 300 python3 -u bench.py --routines dgetrf --extras none --steps 1 --warmup 1 > $O/lu_$nt.txt 2> $O/lu_$nt.err || { tail -20 $O/lu_$nt.err; exit 1; }
  echo "1-GPU nt=$nt: $(grep -E 'timed|backward' $O/lu_$nt.err | tr '\n' ' ')"
done
