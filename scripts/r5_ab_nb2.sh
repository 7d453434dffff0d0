#!/bin/bash
# confirmation: dpotrf nb 1024 vs 1536, dgeqrf nb 512 vs 1024 (1 warm + 2 timed, interleaved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_abnb2; mkdir -p $O
for i in 1 2; do
  for cfg in "dpotrf=1024" "dpotrf=1536" "dgeqrf=512" "dgeqrf=1024"; do
    r=${cfg%%=*}
    timeout -k 10 200 python3 -u bench.py --routines $r --extras none --nb-per $cfg --steps 2 --warmup 1 > $O/$cfg.$i.json 2> $O/$cfg.$i.err || exit 1
    echo "$cfg #$i: $(grep -E 'timed|backward' $O/$cfg.$i.err | sed 's/# //' | tr '\n' ' ')"
  done
done
