#!/bin/bash
# Round 6: one-GPU Cholesky tail width (SLATE_POTRF_TAIL) at n = 65536 / nb 1536 and config 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_potrf_tail; mkdir -p $O
i=0
for rep in 1 2; do
  for t in 4096 2048 6144 8192; do
    i=$((i+1))
    SLATE_POTRF_TAIL=$t timeout -k 10 200 python3 -u bench.py --routines dpotrf --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 --steps 1 --warmup 1 > $O/r$i.txt 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
    echo "tail=$t: $(grep -E 'timed' $O/r$i.err | sed -E 's/# ([a-z0-9_]+) step [0-9]+ timed: ([0-9.]+) ms ([0-9.]+) TFLOP.*/\1 \2 ms \3/' | tr '\n' ' ')"
  done
done
