#!/bin/bash
# Mid-round: traces at the exact bench configs, isolated LU panel sequence,
# critical-path model with the CholeskyQR panel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r4_trace.sh mid && bash scripts/r4_lu_panel_prof.sh && CP_ARGS="--routines lu,qr,chol" bash scripts/r4_critpath.sh
