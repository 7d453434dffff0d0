#!/bin/bash
# isolated panel kernel traces (tournament LU 2048x1024, QR 2048x512) + dgesv_mixed phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/iso; mkdir -p $O
for p in tournament:1024 geqrf:512; do
  name=${p%%:*}; nb=${p##*:}
  PANELS=$name timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$name -o run -- python3 scripts/bench_panel.py 2048 $nb > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  DB=$(find $O/$name -name "*.db" | head -1)
  echo "== $name"; python3 scripts/prof_summary.py $DB 25 | tee $O/${name}_summary.txt
  python3 scripts/tailwin.py $DB --from-end-ms 2 --ms 2 > $O/${name}_win.txt; head -60 $O/${name}_win.txt
  rm -f $DB
done
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 1 --warmup 1 --extras none > $O/gesv_mixed.log 2>&1 || { tail -20 $O/gesv_mixed.log; exit 1; }
grep -E "timed|iters|error" $O/gesv_mixed.log
