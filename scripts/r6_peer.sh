#!/bin/bash
# Round 6: copy-engine peer broadcast (SLATE_BCAST=peer) on the shared-GPU RCCL
# rig + rank 0 under rocprofv3 (kernel + memory-copy trace), multi-device GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_peer; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -k "bcast_modes and peer" > $O/pytest_peer.txt 2>&1 || { tail -60 $O/pytest_peer.txt; exit 1; }
tail -5 $O/pytest_peer.txt
# one traced LU / QR / Cholesky run: rank 0 profiled, 2x2 grid, peer vs rccl
for mode in peer rccl; do
  SLATE_BCAST=$mode SLATE_BCAST_VERBOSE=1 RANK_LOGDIR=$O/ranks_$mode RANK0_WRAP="rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$mode -o r0 --" \
    timeout -k 10 400 python3 scripts/rccl_multi.py 4 getrf_tntpiv,geqrf,potrf --type d --dim 3072 --nb 256 --grid 2x2 --target d --lookahead 2 > $O/rig_$mode.txt 2>&1 || { tail -30 $O/rig_$mode.txt; exit 1; }
  grep -E "all tests|FAIL" $O/rig_$mode.txt | head -3
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "multi_device or from_devices or inproc_allreduce" > $O/pytest_multi.txt 2>&1 || { tail -60 $O/pytest_multi.txt; exit 1; }
tail -3 $O/pytest_multi.txt
