#!/bin/bash
# A/B of the fp32 factor of config 5 (dgesv_mixed) under the round-5 knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abmix; mkdir -p $O
for v in base solve2 nosmall base; do
  unset SLATE_SMALL_SOLVE SLATE_GEMM_SMALL
  [ $v = solve2 ] && export SLATE_SMALL_SOLVE=2
  [ $v = nosmall ] && export SLATE_GEMM_SMALL=0
  timeout -k 10 300 python3 -u bench.py --routines dgesv_mixed --extras none --steps 2 --warmup 1 > $O/m_$v.json 2> $O/m_$v.err || exit 1
  echo "$v: $(grep -E 'timed|factor' $O/m_$v.err | tr '\n' ' ' | cut -c1-400)"
done
