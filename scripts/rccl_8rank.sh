#!/bin/bash
# 8 ranks (2 x 4 grid, the N=8 bench layout) on ONE GPU over RCCL with fake
# host ids: native tester on the headline routines, then bench.py incl. extras.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R="gemm,potrf,getrf,getrf_tntpiv,geqrf,gesv_mixed,gels,trsm,herk"
#timeout -k 10 400 python3 scripts/rccl_multi.py 8 $R --type d --dim 1500 --nb 128 --grid 2x4 --target d --lookahead 2 > gpurun_out/rccl_t_2x4.log 2>&1
#rc=$?; echo "tester 2x4 rc=$rc"; grep -E "FAIL|all tests passed|rror" gpurun_out/rccl_t_2x4.log | head -8
#[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
RANK_TIMEOUT=500 timeout -k 10 560 python3 scripts/rccl_multi.py 8 --cmd python3 bench.py --gpus 8 --dim ${BDIM:-4096} --steps 1 --warmup 1 > gpurun_out/rccl_b8.log 2>&1
rc=$?; echo "bench 8 rc=$rc"; grep -E '^\{|timed|rror|skipped' gpurun_out/rccl_b8.log | cut -c1-400 | head -40
exit $rc
