#!/bin/bash
# Cholesky leaf: focused GPU tests, then dpotrf / dgeqrf / cfg2 / cfg4 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_leafbench; mkdir -p $O
bash scripts/r5_leafprobe.sh || exit 1
timeout -k 10 150 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "potrf or gemm or trsm or posv or geqrf or cholqr or gels" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --routines dpotrf,dgeqrf --extras cfg2_dpotrf_n32768_nb512,cfg4_dgeqrf_nb256 > $O/bench.json 2> $O/bench.err
rc=$?; grep -E "TFLOP|timed" $O/bench.err | tail -12; tail -1 $O/bench.json | cut -c1-300; exit $rc
