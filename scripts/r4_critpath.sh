#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_crit; mkdir -p $O
timeout -k 10 500 python3 -u scripts/critpath.py ${CP_ARGS:-} > $O/critpath.txt 2>&1; rc=$?
cat $O/critpath.txt | tail -80
exit $rc
