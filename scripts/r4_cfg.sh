#!/bin/bash
# BASELINE configs 2 and 4 on one GPU (1-GPU proxies).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_cfg; mkdir -p $O
timeout -k 10 300 python3 bench.py --routines dgeqrf --nb-per dgeqrf=256 --steps 2 --warmup 1 --extras none > $O/cfg4.log 2>&1 || { tail $O/cfg4.log; exit 1; }
echo "cfg4 (dgeqrf nb=256, n=65536): $(grep -E 'timed|backward' $O/cfg4.log | tr '\n' ' ' | cut -c1-240)"
timeout -k 10 300 python3 bench.py --routines dpotrf --dim 32768 --nb-per dpotrf=512 --steps 3 --warmup 1 --extras none > $O/cfg2.log 2>&1 || { tail $O/cfg2.log; exit 1; }
echo "cfg2 (dpotrf n=32768 nb=512): $(grep -E 'timed|backward' $O/cfg2.log | tr '\n' ' ' | cut -c1-300)"
