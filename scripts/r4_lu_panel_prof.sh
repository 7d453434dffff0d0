#!/bin/bash
# Kernel sequence of the isolated tournament panel (last repetition) at the
# 2x4 per-GPU shapes: local 32768 x 512, tree merge 1024 x 512.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_lupanel; mkdir -p $O
for MS in "32768 512" "1024 512"; do
  set -- $MS
  PANELS=getrf_tournament timeout -k 10 200 rocprofv3 --kernel-trace -d $O/p_$1_$2 -o run -- python3 scripts/bench_panel.py $1 $2 > $O/p_$1_$2.log 2>&1 || { tail $O/p_$1_$2.log; exit 1; }
  DB=$(find $O/p_$1_$2 -name "*.db" | head -1)
  python3 scripts/panel_seq.py $DB --list > $O/seq_$1_$2.txt 2>&1
  rm -rf $O/p_$1_$2
  grep -E " ms$" $O/p_$1_$2.log; head -24 $O/seq_$1_$2.txt
done
