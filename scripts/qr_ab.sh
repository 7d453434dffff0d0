#!/bin/bash
# A/B of the QR narrow panel: TSQR (default) vs column path; isolated panel + full dgeqrf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_panel.py 65536 512 2>&1 | grep geqrf
SLATE_QR_PANEL=columns timeout -k 10 120 python scripts/bench_panel.py 65536 512 2>&1 | grep geqrf
timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 1 ${BENCH_ARGS:-} 2>&1 | grep timed
SLATE_QR_PANEL=columns timeout -k 10 300 python bench.py --routines dgeqrf --steps 1 --warmup 1 ${BENCH_ARGS:-} 2>&1 | grep timed
