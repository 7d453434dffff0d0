#!/bin/bash
# Round 6: the bench's multi-rank path with the 8-GPU defaults (per-routine
# grids, LU nb 256, SUMMA on the unmasked queue, peer broadcasts) rehearsed as
# 2 / 8 ranks sharing this one GPU at a small n, then the default 1-GPU bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_verify; mkdir -p $O
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --dim 16384 --steps 1 --warmup 1 > $O/b2.txt 2> $O/b2.err || { tail -40 $O/b2.err; exit 1; }
tail -1 $O/b2.txt
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 500 python3 -u bench.py --gpus 8 --dim 8192 --steps 1 --warmup 1 > $O/b8.txt 2> $O/b8.err || { tail -40 $O/b8.err; exit 1; }
tail -1 $O/b8.txt
timeout -k 10 900 python3 -u bench.py > $O/b1.txt 2> $O/b1.err || { tail -40 $O/b1.err; exit 1; }
tail -1 $O/b1.txt
