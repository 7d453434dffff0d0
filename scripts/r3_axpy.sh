#!/bin/bash
# axpy-form small triangular kernels: tests, potrf/getrf benches, isolated traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/axpy; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "trsm or trtri or potrf or posv or potri or getrf or gesv or lu or chol or inv or qr or gels or unmqr" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 bench.py --routines dpotrf,dgetrf,dgeqrf --steps 1 --warmup 1 --extras cfg2_dpotrf_n32768_nb512 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -E "timed|error|cfg2" $O/bench.log | cut -c1-300
bash scripts/r3_iso_prof.sh 2>&1 | grep -v "^W2026" | tail -120
