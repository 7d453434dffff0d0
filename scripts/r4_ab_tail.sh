#!/bin/bash
# A/B of this round's 1-GPU options (potrf tail finish, CholeskyQR p=1 QR panel)
# plus the GPU tests of the new device paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_ab; mkdir -p $O
K="inproc or shared_gpu or 2x4 or no_fast_lane" timeout -k 10 900 bash scripts/r4_gpu_quick.sh || exit $?
for T in 0 4096 8192; do
  SLATE_POTRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dpotrf --dim 32768 --nb-per dpotrf=512 --steps 3 --warmup 1 --extras none > $O/cfg2_tail$T.log 2>&1 || { tail $O/cfg2_tail$T.log; exit 1; }
  echo "cfg2 tail=$T: $(grep -E 'timed|backward' $O/cfg2_tail$T.log | tr '\n' ' ' | cut -c1-400)"
done
for T in 0 4096; do
  SLATE_POTRF_TAIL=$T timeout -k 10 300 python3 bench.py --routines dpotrf --steps 2 --warmup 1 --extras none > $O/potrf_tail$T.log 2>&1 || { tail $O/potrf_tail$T.log; exit 1; }
  echo "potrf64k tail=$T: $(grep -E 'timed|backward' $O/potrf_tail$T.log | tr '\n' ' ' | cut -c1-400)"
done
for C in 0 1; do
  SLATE_QR_CHOLQR1=$C timeout -k 10 300 python3 bench.py --routines dgeqrf --steps 2 --warmup 1 --extras none > $O/qr_cq$C.log 2>&1 || { tail $O/qr_cq$C.log; exit 1; }
  echo "dgeqrf cholqr1=$C: $(grep -E 'timed|backward' $O/qr_cq$C.log | tr '\n' ' ' | cut -c1-400)"
done
