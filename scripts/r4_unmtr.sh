#!/bin/bash
# Blocked one-process unmtr_he2hb (SLATE_UNMTR_GROUP) A/B + GPU heev tests,
# then the BASELINE config 2 / 4 one-GPU proxies.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4_unmtr; mkdir -p $O
SLATE_UNMTR_GROUP=4 K="heev or hegv or eig or stedc" bash scripts/r4_gpu_quick.sh || exit 1
for G in 4 1 4 1; do  # default 1 until this A/B
  SLATE_UNMTR_GROUP=$G EIG_PROF_OUT=$O timeout -k 10 300 python3 -u scripts/eig_prof.py 8192 256 d heev > $O/heev_g$G.log 2>&1 || { tail $O/heev_g$G.log; exit 1; }
  echo "== group=$G"; grep -E "^heev|unmtr_he2hb|residual" $O/heev_g$G.log
done
bash scripts/r4_cfg.sh
