#!/bin/bash
# Round 6: fp32 512-thread tournament trees (two rows per thread, <= 256 VGPRs): correctness,
# isolated fp32 panels 256 vs 512, the 2-rank rig's config 5 with the reserved-CU default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_f32_nt; mkdir -p $O
SLATE_TSLU_NT=512 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "tournament or tntpiv or mixed" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for nt in 256 512 256 512; do
  for mn in "32768 512" "32768 256" "1024 512"; do
    DTYPE=float32 SLATE_TSLU_NT=$nt PANELS=tournament timeout -k 10 120 python3 -u scripts/bench_panel.py $mn 2>&1 | grep getrf | sed "s/^/fp32 nt=$nt /" | tee -a $O/panels.txt || exit 1
  done
done
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 500 python3 -u bench.py --gpus 2 --dim 16384 --routines none --extras cfg5_dgesv_mixed,cfg3_dgetrf_tntpiv_nb512 --extras-steps 1 > $O/b2.txt 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
grep -E "backward|phase" $O/b2.err
