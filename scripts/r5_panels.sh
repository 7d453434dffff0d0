#!/bin/bash
# LU tournament panel (local 32768 x 512, merge-sized 1024 x 512) and lu_sign:
# isolated timings + per-kernel composition of one panel; then the 2x4 model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_panels; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py tests/test_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lu_sign or geqrf or cholqr or potrf_leaf or potrf_kernel or gels or tsqr" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r5_leafprobe.sh || exit 1
for MS in "32768 512" "1024 512"; do
  set -- $MS
  PANELS=getrf_tournament timeout -k 10 120 python3 scripts/bench_panel.py $1 $2 2>&1 | grep ms || exit 1
  PANELS=getrf_tournament timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_$1 -o run -- python3 scripts/bench_panel.py $1 $2 > /dev/null 2>&1 || exit 1
  DB=$(find $O/p_$1 -name "*.db" | head -1); python3 scripts/panel_seq.py $DB > $O/seq_$1.txt 2>&1; sed -n '/group 2/,$p' $O/seq_$1.txt | head -16
done
timeout -k 10 120 python3 scripts/lusign_probe.py 256,512,1024 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_lusign -o run -- python3 scripts/lusign_probe.py 512 > /dev/null 2>&1 || exit 1
DB=$(find $O/p_lusign -name "*.db" | head -1); python3 scripts/panel_seq.py $DB > $O/seq_lusign.txt 2>&1; sed -n '/group 2/,$p' $O/seq_lusign.txt | head -16
timeout -k 10 500 python3 -u scripts/critpath.py --p 2 --q 4 --every 16 --reps 2 > $O/crit_2x4.txt 2>&1 || { tail -20 $O/crit_2x4.txt; exit 1; }
grep -E "==|steps whose|predicted" $O/crit_2x4.txt
