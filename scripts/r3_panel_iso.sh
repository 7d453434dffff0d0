#!/bin/bash
# device panels in isolation across M (tournament LU nb=1024, QR nb=512) + kernel trace of the small-M ones
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/panel_iso; mkdir -p $O
for m in 2048 8192 32768; do
  timeout -k 10 120 python3 scripts/bench_panel.py $m 1024 >> $O/panel.txt 2>&1 || { tail -20 $O/panel.txt; exit 1; }
done
for m in 2048 8192 32768; do
  timeout -k 10 120 python3 scripts/bench_panel.py $m 512 >> $O/panel.txt 2>&1 || { tail -20 $O/panel.txt; exit 1; }
done
grep -v "^W2026\|amdgpu.ids" $O/panel.txt
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 scripts/bench_panel.py 2048 1024 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
DB=$(find $O/tr -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 40 > $O/summary_2048.txt; cat $O/summary_2048.txt
python3 scripts/tailwin.py $DB --from-end-ms 30 --ms 30 > $O/win_2048.txt; head -80 $O/win_2048.txt
rm -f $DB
