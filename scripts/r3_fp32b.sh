#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fp32b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "trsm or getrf or gesv or tournament" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 1; }
grep -E "timed|iters|backward" $O/g.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 bench.py --routines dgesv_mixed --steps 1 --warmup 0 --extras none --check no > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
DB=$(find $O/tr -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 16 > $O/summary.txt; python3 scripts/timeline.py $DB >> $O/summary.txt; cat $O/summary.txt
rm -f $DB
