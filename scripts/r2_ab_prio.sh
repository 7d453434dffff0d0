#!/bin/bash
# A/B of the panel-kernel wave priority (s_setprio, SLATE_PANEL_PRIO): the tree's
# build (priority on) against alt/ (same sources built with SLATE_PANEL_PRIO=0),
# interleaved on one box; device kernel tests of the priority build first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abprio
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 > gpurun_out/abprio/tests.log 2>&1 || { tail -20 gpurun_out/abprio/tests.log; exit 1; }
tail -1 gpurun_out/abprio/tests.log
ARGS="--routines dpotrf,dgetrf,dgeqrf --steps 1 --warmup 1 --extras cfg2_dpotrf_n32768_nb512 --extras-steps 2 --check no"
for v in prio noprio prio2 noprio2; do
  B=bench.py; case $v in noprio*) B=alt/bench.py;; esac
  timeout -k 10 200 python $B $ARGS > gpurun_out/abprio/$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/abprio/$v.log; exit 1; }
  echo "$v: $(grep -h 'timed' gpurun_out/abprio/$v.log | grep -v 'step 1 timed.*cfg2' | tr '\n' ' ')"
done
