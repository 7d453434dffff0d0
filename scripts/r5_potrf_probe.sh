#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_pp; mkdir -p $O
timeout -k 10 120 python3 scripts/potrf_diag_probe.py 2>&1 | grep potrf
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p -o run -- python3 scripts/potrf_diag_probe.py 512 > /dev/null 2>&1 || exit 1
DB=$(find $O/p -name "*.db" | head -1); python3 scripts/panel_seq.py $DB --list 2>&1 | head -30
