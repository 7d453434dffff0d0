#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/perm2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "wide_tiles or getrf or permute or gesv" > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
tail -1 $O/p1.log
timeout -k 10 900 python -u -m pytest tests/test_dist.py -x -q --timeout 600 --timeout-method thread -k "rccl_lu_qr_p_gt_1 or rccl_2x4" > $O/p2.log 2>&1 || { tail -30 $O/p2.log; exit 1; }
tail -1 $O/p2.log
for r in 1 2; do timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/g.log 2>&1 || exit 1; grep -E "timed|backward" $O/g.log; done
