#!/bin/bash
# end-of-round: full GPU suite + smoke, then the 2x4 critical-path model
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/r5_suite.sh || exit 1
O=gpurun_out/r5_end; mkdir -p $O
timeout -k 10 400 python3 -u scripts/critpath.py --p 2 --q 4 --every 16 --reps 2 > $O/crit_2x4.txt 2>&1 || { tail -20 $O/crit_2x4.txt; exit 1; }
grep -E "==|steps whose|predicted" $O/crit_2x4.txt
