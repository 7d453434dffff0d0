#!/bin/bash
# Round 6: NN GEMMs with K in (1000, 2048] and m, n >= 8192 as TN on a packed A
# (default) vs NT on a copied B (SLATE_GEMM_PACK_A_MINK=2048, round 5): 1-GPU bench + SUMMA model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_packa; mkdir -p $O
for mk in 2048 1000 2048 1000; do
  SLATE_GEMM_PACK_A_MINK=$mk timeout -k 10 400 python3 -u bench.py --extras cfg2_dpotrf_n32768_nb512,cfg4_dgeqrf_nb256 --extras-steps 1 --steps 1 --warmup 1 > $O/b_$mk.txt 2> $O/b_$mk.err || { tail -20 $O/b_$mk.err; exit 1; }
  echo "mink=$mk: $(grep -E 'timed' $O/b_$mk.err | sed -E 's/# ([a-z0-9_]+) step [0-9]+ timed: ([0-9.]+) ms ([0-9.]+) TFLOP.*/\1 \3/' | tr '\n' ' ') value $(tail -1 $O/b_$mk.txt | sed -E 's/.*"value": ([0-9.]+).*/\1/')"
done
for mk in 2048 1000; do
  SLATE_GEMM_PACK_A_MINK=$mk SLATE_PANEL_CUS=32 timeout -k 10 120 python3 -u scripts/critpath.py --p 2 --q 4 --nb 512 --summa-k 2048 --reps 2 --routines gemm 2>&1 | grep "== dgemm" | sed "s/^/mink=$mk /" || exit 1
done
