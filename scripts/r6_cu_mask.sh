#!/bin/bash
# Round 6: XCD-balanced CU reservation.  (1) placement + complement-mask GEMM
# rate probe; (2) 1-GPU A/B of SLATE_PANEL_CUS / mode, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_cumask; mkdir -p $O
timeout -k 10 120 ./tools_bin/cu_mask_probe 8 16 24 32 > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for cfg in ${CFGS:-0:shared 8:shared 16:shared 32:shared 16:exclusive 0:shared 16:shared}; do
  v=${cfg%%:*}; mode=${cfg##*:}
  export SLATE_PANEL_CUS=$v SLATE_PANEL_CUS_MODE=$mode
  timeout -k 10 300 python3 -u bench.py --routines ${ROUTINES:-dpotrf,dgetrf,dgeqrf} --extras ${EXTRAS:-cfg2_dpotrf_n32768_nb512} --steps 1 --warmup 1 --check no > $O/c_${v}_$mode.json 2> $O/c_${v}_$mode.err || exit 1
  echo "cus=$v $mode: $(grep timed $O/c_${v}_$mode.err | sed 's/# //; s/ step 1 timed//' | tr '\n' ' ')"
done
