#!/bin/bash
# Round 6: config-5 fp32 factor (dgesv_mixed n=65536) vs CU reservation and tournament version
# (cfg = panel CUs : SLATE_TSLU : SLATE_TSLU_F32_R)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_cfg5; mkdir -p $O
for cfg in ${CFGS:-0:1:4 0:2:4 0:2:2 32:2:2 32:1:4 0:1:4}; do
  IFS=: read R V F <<< "$cfg"
  SLATE_PANEL_CUS=$R SLATE_TSLU=$V SLATE_TSLU_F32_R=$F timeout -k 10 300 python3 -u bench.py --routines none --extras cfg5_dgesv_mixed --extras-steps 1 --extras-warmup 1 --check no > $O/c_${R}_${V}_$F.json 2> $O/c_${R}_${V}_$F.err || exit 1
  echo "cus=$R tslu=v$V f32R=$F: $(grep -E 'timed|phase ms' $O/c_${R}_${V}_$F.err | tail -2 | tr '\n' ' ' | cut -c1-260)"
done
