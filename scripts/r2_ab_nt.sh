#!/bin/bash
# A/B of the NT trailing-update form (SLATE_UPDATE_NT) for dgetrf / dgeqrf at
# n=65536 on one GPU, device tests of both paths, then a kernel trace of
# dpotrf at the BASELINE config-2 size (n=32768, nb=512).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abnt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 -k "getrf or geqrf or gesv or gels" > gpurun_out/abnt/tests.log 2>&1 || { tail -20 gpurun_out/abnt/tests.log; exit 1; }
tail -1 gpurun_out/abnt/tests.log
for nt in 1 0; do
  SLATE_UPDATE_NT=$nt timeout -k 10 200 python bench.py --routines dgetrf,dgeqrf --steps 1 --warmup 1 --extras none --check yes > gpurun_out/abnt/nt$nt.log 2>&1 || { echo "nt=$nt FAILED"; tail -5 gpurun_out/abnt/nt$nt.log; exit 1; }
  echo "NT=$nt: $(grep -h -e 'step 1 timed' -e backward gpurun_out/abnt/nt$nt.log | tr '\n' ' ')"
done
R=dpotrf N=32768 BENCH_ARGS="--nb 512" O=abnt/potrf32k bash scripts/prof_qr.sh
