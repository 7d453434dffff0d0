#!/bin/bash
# Round 6: 1-GPU bench A/B of SE-balanced CU reservation after the null-stream fix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_cusb; mkdir -p $O
for cfg in ${CFGS:-0:1 32:1 32:0 64:1 0:1 32:1}; do
  v=${cfg%%:*}; la=${cfg##*:}
  export SLATE_PANEL_CUS=$v SLATE_PANEL_CUS_LA=$la
  timeout -k 10 300 python3 -u bench.py --routines ${ROUTINES:-dpotrf,dgetrf,dgeqrf} --extras ${EXTRAS:-cfg2_dpotrf_n32768_nb512} --steps 1 --warmup 1 --check no > $O/c_${v}_$la.json 2> $O/c_${v}_$la.err || exit 1
  echo "cus=$v la_masked=$la: $(grep timed $O/c_${v}_$la.err | sed 's/# //; s/ step 1 timed//' | tr '\n' ' ')"
done
