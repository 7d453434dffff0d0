#!/bin/bash
# A/B: TSQR tree kernels (qr_node / qr_node_q) with and without the panel wave
# priority; tree build = priority on, alt/ = SLATE_QR_NODE_PRIO=0; interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abqrn
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 280 -k "gemm or geqrf or gels or norm" > gpurun_out/abqrn/tests.log 2>&1 || { tail -30 gpurun_out/abqrn/tests.log; exit 1; }
tail -1 gpurun_out/abqrn/tests.log
for v in on off on2 off2; do
  B=bench.py; case $v in off*) B=alt/bench.py;; esac
  timeout -k 10 200 python $B --routines dgeqrf --steps 2 --warmup 1 --extras none --check no > gpurun_out/abqrn/$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/abqrn/$v.log; exit 1; }
  echo "$v: $(grep -h 'timed' gpurun_out/abqrn/$v.log | tr '\n' ' ')"
done
