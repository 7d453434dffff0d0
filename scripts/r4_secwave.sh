#!/bin/bash
# Wave-per-root secular kernel: GPU eigen tests, heev A/B (SLATE_SECULAR_WAVE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_secwave; mkdir -p $O
K="stedc or heev or hegv or eig" bash scripts/r4_gpu_quick.sh || exit 1
for W in 1 0 1 0; do
  SLATE_SECULAR_WAVE=$W EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_w$W.log 2>&1 || { tail $O/heev_w$W.log; exit 1; }
  echo "== wave=$W"; grep -E "^heev|stedc_dist|stedc_m_secular|residual" $O/heev_w$W.log
done
