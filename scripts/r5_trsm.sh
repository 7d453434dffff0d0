#!/bin/bash
# trsm_small on the leaf_solve stream: focused tests, LU panel timings + composition
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_trsm; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "trsm or getrf or tournament or gesv or lu_sign or potrf_leaf or getrs" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for MS in "32768 512" "1024 512"; do
  set -- $MS
  PANELS=getrf_tournament timeout -k 10 120 python3 scripts/bench_panel.py $1 $2 2>&1 | grep ms || exit 1
  PANELS=getrf_tournament timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_$1 -o run -- python3 scripts/bench_panel.py $1 $2 > /dev/null 2>&1 || exit 1
  DB=$(find $O/p_$1 -name "*.db" | head -1); python3 scripts/panel_seq.py $DB > $O/seq_$1.txt 2>&1; sed -n '/group 2/,$p' $O/seq_$1.txt | head -14
done
