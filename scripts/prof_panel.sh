#!/bin/bash
# kernel trace of the isolated geqrf panel (65536 x 512) -> per-kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof_panel; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O -o run -- python3 scripts/bench_panel.py ${M:-65536} ${NB:-512} > $O/log.txt 2>&1 || exit $?
grep geqrf $O/log.txt
DB=$(find $O -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 25
rm -f $DB
