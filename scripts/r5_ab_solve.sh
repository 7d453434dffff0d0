#!/bin/bash
# A/B: round-4 small triangular solves (SLATE_SMALL_SOLVE=1) vs the solve-stream ones, in situ
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_ab; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "trsm or getrf or tournament or gesv or trtri or inverse or getri" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new v1 new v1; do
  if [ $v = v1 ]; then export SLATE_SMALL_SOLVE=1; else unset SLATE_SMALL_SOLVE; fi
  timeout -k 10 300 python3 -u bench.py --routines dgetrf --extras none --steps 2 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  echo "$v: $(grep timed $O/b_$v.err | tr '\n' ' ')"
done
