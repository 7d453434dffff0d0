#!/bin/bash
# GPU tests + bench sweep over SLATE_PANEL_CUS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for cus in ${CUS_LIST:-0 32}; do
  SLATE_PANEL_CUS=$cus timeout -k 10 600 python bench.py ${BENCH_ARGS:---routines dpotrf,dgetrf,dgeqrf --n 32768 --steps 1 --warmup 1} > gpurun_out/bench_cus$cus.log 2>&1 || exit $?
  echo "== SLATE_PANEL_CUS=$cus"; grep "^#" gpurun_out/bench_cus$cus.log | grep timed; tail -1 gpurun_out/bench_cus$cus.log | cut -c1-400
done
