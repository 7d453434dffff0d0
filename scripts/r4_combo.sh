#!/bin/bash
# Round-4 combined validation: QR split-K / CholQR panel, stage-2 sliding
# window A/B, heev / svd timings, dgeqrf bench, QR critical path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_combo; mkdir -p $O
K="${K:-herk_kernel or geqrf or gels or stage2_fused or heev_device or svd_device or shared_gpu}" bash scripts/r4_gpu_quick.sh || exit 1
timeout -k 10 200 python3 -u scripts/bench_cholqr.py 32768 4096 > $O/cq.log 2>&1 && grep mr= $O/cq.log || exit 1
for S in 1 0; do
  SLATE_HB2ST_SLIDE=$S EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_slide$S.log 2>&1 || { tail $O/heev_slide$S.log; exit 1; }
  echo "== slide=$S"; grep -v "^W20\|amdgpu.ids" $O/heev_slide$S.log | head -24
done
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d svd > $O/svd.log 2>&1; grep -v "^W20\|amdgpu.ids" $O/svd.log | head -26
SLATE_EIG_KD=32 EIG_PROF_OUT=$O timeout -k 10 400 python3 -u scripts/eig_prof.py 8192 256 d heev,svd > $O/eig_kd32.log 2>&1; echo "== kd=32"; grep -E "^(heev|svd)|hb2st|tb2bd|bdsqr |he2hb|ge2tb|unmtr_hb2st_fused" $O/eig_kd32.log | head -20
timeout -k 10 300 python3 bench.py --routines dgeqrf --steps 2 --warmup 1 --extras none > $O/dgeqrf.log 2>&1 && grep -E "timed|backward" $O/dgeqrf.log || exit 1
CP_ARGS="--routines qr" bash scripts/r4_critpath.sh
