#!/bin/bash
# gemv chunking for the refinement solves (cfg5), 8-rank 2x4 RCCL rig bench
# with the multi-GPU defaults (lookahead 2), quick device tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_mix; mkdir -p $O
K="${K:-gemv or trsm_kernel or mixed or gesv or factor}" bash scripts/r4_gpu_quick.sh || exit 1
timeout -k 10 300 python3 bench.py --routines dgesv_mixed --steps 2 --warmup 1 --extras none > $O/cfg5.log 2>&1 && grep -E "timed|phase|backward" $O/cfg5.log || exit 1
BDIM=4096 bash scripts/rccl_8rank.sh
EIG_PROF_OUT=gpurun_out/r4_mix timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > gpurun_out/r4_mix/heev.log 2>&1; grep -E "^heev|stedc" gpurun_out/r4_mix/heev.log
