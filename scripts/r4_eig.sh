#!/bin/bash
# Fused stage-2 back-transform: GPU tests, then heev / svd stage timings at
# n = 8192 with the fused kernels and with the blocked GEMM sequence (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_eig; mkdir -p $O
K="${K:-stage2_fused or heev_device or svd_device or geqrf}" bash scripts/r4_gpu_quick.sh || exit 1
for F in 1 0; do
  SLATE_HB2ST_FUSED=$F EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev,svd > $O/eig_fused$F.log 2>&1 || { tail -20 $O/eig_fused$F.log; exit 1; }
  echo "== fused=$F"; grep -E "^(heev|svd)|unmtr|hb2st|tb2bd|bdsqr|stedc|he2hb|ge2tb|unmbr" $O/eig_fused$F.log | head -40
done
timeout -k 10 300 python3 bench.py --routines dgeqrf --steps 2 --warmup 1 --extras none > $O/dgeqrf.log 2>&1 && grep -E "timed|backward" $O/dgeqrf.log
SLATE_GETRF_TAIL=2048 timeout -k 10 300 python3 -u scripts/getrf_tail_check.py > $O/tail_check.log 2>&1; rc=$?; tail -12 $O/tail_check.log; [ $rc = 0 ] || exit 1
for T in 0 4096 8192; do
  SLATE_GETRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dgetrf --steps 2 --warmup 1 --extras none > $O/getrf_tail$T.log 2>&1 || { tail $O/getrf_tail$T.log; exit 1; }
  echo "dgetrf tail=$T: $(grep -E 'timed|backward' $O/getrf_tail$T.log | tr '\n' ' ')"
done
for T in 0 4096; do
  SLATE_GETRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none > $O/mixed_tail$T.log 2>&1 || { tail $O/mixed_tail$T.log; exit 1; }
  echo "gesv_mixed tail=$T: $(grep -E 'timed|phase|backward' $O/mixed_tail$T.log | tr '\n' ' ')"
done
