#!/bin/bash
# A/B previous commit (abprev/) vs working tree, plus tests of the changed kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "trsm or trtri or potrf or posv or potri or getrf or gesv or lu or chol or inv or qr or gels or unmqr or tournament" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in abprev .; do
    timeout -k 10 400 python3 $v/bench.py --routines dgetrf,dgeqrf --steps 1 --warmup 1 --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 --check no > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "== $v"; grep -E "step 1 timed" $O/b.log
  done
done
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none --check no > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 1; }
echo "== gesv_mixed"; grep -E "timed|iters" $O/g.log | cut -c1-160
