#!/bin/bash
# dgesv_mixed (fp32 tntpiv factor) tile width / lookahead / tail sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_mixed_nb; mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none ${ARGS} > $O/$name.log 2>&1 || { tail $O/$name.log; return 1; }
  echo "$name: $(grep -E 'phase|timed' $O/$name.log | tr '\n' ' ' | cut -c1-420)"
}
ARGS="--nb-per dgesv_mixed=1024" run nb1024 SLATE_X=0 || exit 1
ARGS="--nb-per dgesv_mixed=2048" run nb2048 SLATE_X=0 || exit 1
ARGS="--nb-per dgesv_mixed=1024 --lookahead 2" run nb1024_la2 SLATE_X=0 || exit 1
ARGS="--nb-per dgesv_mixed=768" run nb768 SLATE_X=0 || exit 1
ARGS="--nb-per dgesv_mixed=1024" run nb1024_tail8192 SLATE_GETRF_TAIL=8192 || exit 1
