#!/bin/bash
# Multi-rank RCCL validation on one GPU (fake host ids): native tester on 1x2, 2x1, 2x2
# grids, then the headline bench on 2 and 4 ranks at a small size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R="gemm,herk,trsm,trmm,potrf,posv,getrf,getrf_tntpiv,getrf_nopiv,gesv,geqrf,gelqf,gels,gesv_mixed,posv_mixed,heev,svd,hesv,getri,trtri,genorm"
for g in "2 1x2" "2 2x1" "4 2x2"; do
  set -- $g
  timeout -k 10 400 python3 scripts/rccl_multi.py $1 $R --type d,z --dim 700 --nb 128 --grid $2 --target d > gpurun_out/rccl_t_$2.log 2>&1
  rc=$?; echo "tester $2 rc=$rc"; grep -E "FAIL|all tests passed|rror" gpurun_out/rccl_t_$2.log | head -8
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for n in 2 4; do
  timeout -k 10 400 python3 scripts/rccl_multi.py $n --cmd python3 bench.py --gpus $n --dim ${BDIM:-16384} --steps 1 --warmup 1 > gpurun_out/rccl_b$n.log 2>&1
  rc=$?; echo "bench $n rc=$rc"; grep -E '^\{|timed|rror' gpurun_out/rccl_b$n.log | cut -c1-300 | head -8
  [ $rc -ne 0 ] && exit $rc
done
exit 0
