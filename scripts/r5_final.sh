#!/bin/bash
# focused tests + full default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_final; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "trsm or getrf or tournament or gesv or trtri or potrf or lu_sign or geqrf" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; grep -E "timed" $O/bench.err | tail -24; tail -1 $O/bench.json | cut -c1-200; exit $rc
