#!/bin/bash
# Round-4 kernel traces at the exact bench configs (1 GPU): dgetrf nb 2048,
# dgeqrf nb 512, dpotrf nb 1024, config 2 (dpotrf n 32768 nb 512), fp32 LU of
# dgesv_mixed.  Usage: r4_trace.sh <tag> [routine-specs...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-start}; shift
O=gpurun_out/r4_$TAG; mkdir -p $O
SPECS=${@:-"dgetrf dgeqrf dpotrf cfg2 fp32lu"}
for S in $SPECS; do
  case $S in
    cfg2)   ARGS="--routines dpotrf --dim 32768 --nb-per dpotrf=512" ;;
    fp32lu) ARGS="--routines dgesv_mixed" ;;
    *)      ARGS="--routines $S" ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$S -o run -- python3 bench.py $ARGS --steps 1 --warmup 1 --extras none --check no > $O/$S.log 2>&1 || { tail -20 $O/$S.log; exit 1; }
  DB=$(find $O/$S -name "*.db" | head -1)
  { grep -E "timed|phase" $O/$S.log; python3 scripts/prof_summary.py $DB 20; python3 scripts/timeline.py $DB; python3 scripts/steps.py $DB --last 12; } > $O/trace_$S.txt 2>&1
  rm -rf $O/$S
  head -4 $O/trace_$S.txt
done
