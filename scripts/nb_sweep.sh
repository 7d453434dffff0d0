#!/bin/bash
# nb sweep of single routines at the bench size: NB_LIST="dgetrf:768 dpotrf:1024 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rn in ${NB_LIST:-dgetrf:512 dgetrf:768 dgetrf:1024}; do
  r=${rn%%:*}; nb=${rn##*:}
  timeout -k 10 300 python bench.py --routines $r --nb $nb --steps 1 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/nb_${r}_$nb.log 2>&1 || exit $?
  echo "$r nb=$nb $(grep timed gpurun_out/nb_${r}_$nb.log)"
done
