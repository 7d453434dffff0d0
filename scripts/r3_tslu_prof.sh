#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tslu_prof; mkdir -p $O
for mode in 0 1; do
  SLATE_TSLU_WG=$mode PANELS=tournament timeout -k 10 120 rocprofv3 --kernel-trace -d $O/m$mode -o run -- python3 scripts/bench_panel.py ${M:-2048} 1024 > $O/m$mode.log 2>&1 || { tail -20 $O/m$mode.log; exit 1; }
  DB=$(find $O/m$mode -name "*.db" | head -1)
  echo "== wg=$mode"; python3 scripts/prof_summary.py $DB 20
  python3 scripts/tailwin.py $DB --from-end-ms 3 --ms 3 | head -70
  rm -f $DB
done
