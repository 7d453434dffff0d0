#!/bin/bash
# Round 6 final: critical-path model at the 8-GPU bench defaults (32 reserved CUs,
# CU-free peer messages): LU 2x4 nb 512, QR 8x1 nb 512, Cholesky 4x2 nb 512,
# SUMMA dgemm 2x4 K = 2048 on the unmasked queue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_critpath_final; mkdir -p $O
SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 2 --q 4 --nb 512 --every 16 --reps 2 --routines lu > $O/lu.txt 2>&1 || { tail -5 $O/lu.txt; exit 1; }
SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 8 --q 1 --nb 512 --every 16 --reps 2 --routines qr > $O/qr.txt 2>&1 || { tail -5 $O/qr.txt; exit 1; }
SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 4 --q 2 --nb 512 --every 16 --reps 2 --routines chol > $O/chol.txt 2>&1 || { tail -5 $O/chol.txt; exit 1; }
SLATE_PANEL_CUS=0 timeout -k 10 200 python3 -u scripts/critpath.py --p 2 --q 4 --nb 512 --summa-k 2048 --reps 2 --routines gemm > $O/gemm.txt 2>&1 || { tail -5 $O/gemm.txt; exit 1; }
grep -hE "^==|sampled sums|CU-free messages" $O/lu.txt $O/qr.txt $O/chol.txt $O/gemm.txt
