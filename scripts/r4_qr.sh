#!/bin/bash
# Split-K Gram matrix for the CholeskyQR panel: kernel tests, isolated pass
# pieces, dgeqrf bench, p x q critical-path model (QR).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_qr; mkdir -p $O
K="${K:-herk_kernel or geqrf or gels or heev_device or svd_device or shared_gpu}" bash scripts/r4_gpu_quick.sh || exit 1
timeout -k 10 200 python3 -u scripts/bench_cholqr.py 32768 4096 > $O/cq.log 2>&1 && grep mr= $O/cq.log || exit 1
timeout -k 10 300 python3 bench.py --routines dgeqrf --steps 2 --warmup 1 --extras none > $O/dgeqrf.log 2>&1 && grep -E "timed|backward" $O/dgeqrf.log || exit 1
EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev,svd > $O/eig.log 2>&1; grep -E "^(heev|svd)|unmtr|hb2st|tb2bd|bdsqr|stedc_dist|he2hb|ge2tb" $O/eig.log | head -30
CP_ARGS="--routines qr" bash scripts/r4_critpath.sh
