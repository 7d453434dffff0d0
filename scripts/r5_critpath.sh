#!/bin/bash
# Critical-path model: chain alone, update alone, and the contended step (chain on the
# panel queue while the trailing GEMM runs) at 2x4 (the 8-GPU headline geometry) and
# at 1x1 with the bench's tile sizes (sanity check against the driver-timed 1-GPU numbers).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_crit; mkdir -p $O
timeout -k 10 500 python3 -u scripts/critpath.py --p 2 --q 4 --every 16 --reps 2 > $O/crit_2x4.txt 2>&1 || { tail -20 $O/crit_2x4.txt; exit 1; }
grep -E "==|steps whose|predicted" $O/crit_2x4.txt
timeout -k 10 300 python3 -u scripts/critpath.py --p 1 --q 1 --nb 2048 --every 4 --reps 2 --routines lu > $O/crit_1x1_lu.txt 2>&1 || { tail -20 $O/crit_1x1_lu.txt; exit 1; }
timeout -k 10 300 python3 -u scripts/critpath.py --p 1 --q 1 --nb 1024 --every 8 --reps 2 --routines chol > $O/crit_1x1_chol.txt 2>&1 || { tail -20 $O/crit_1x1_chol.txt; exit 1; }
timeout -k 10 300 python3 -u scripts/critpath.py --p 1 --q 1 --nb 512 --every 16 --reps 2 --routines qr,gemm > $O/crit_1x1_qr.txt 2>&1 || { tail -20 $O/crit_1x1_qr.txt; exit 1; }
grep -E "==|steps whose|predicted" $O/crit_1x1_*.txt
