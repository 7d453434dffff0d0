#!/bin/bash
# Round 6 final: 8 ranks on the shared-GPU rig, n = 8192, every extra config, final defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_b8_final; mkdir -p $O
( while sleep 50; do echo "hb $(date +%T)"; done ) &
hb=$!
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 800 python3 -u bench.py --gpus 8 --dim 8192 --steps 1 --warmup 1 > $O/b.txt 2> $O/b.err
rc=$?
kill $hb
grep -E "backward|skipped" $O/b.err
exit $rc
