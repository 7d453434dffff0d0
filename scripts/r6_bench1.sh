#!/bin/bash
# Round 6 final: the default 1-GPU bench (what the driver runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_bench1; mkdir -p $O
timeout -k 10 900 python3 -u bench.py > $O/b1.txt 2> $O/b1.err || { tail -40 $O/b1.err; exit 1; }
tail -1 $O/b1.txt | cut -c1-400
