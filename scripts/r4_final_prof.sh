#!/bin/bash
# End-of-round evidence: kernel traces at the exact bench configs, the p x q
# critical-path model, svd kernel trace (bdsqr rotations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/r4_trace.sh final ${SPECS:-dgetrf dgeqrf dpotrf cfg2 fp32lu} || exit 1
CP_ARGS="--routines lu,qr,chol" bash scripts/r4_critpath.sh | tail -60 || exit 1
O=gpurun_out/r4_final; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/svd -o run -- python3 scripts/eig_prof.py 8192 256 d svd > $O/svd_prof.log 2>&1 || { tail $O/svd_prof.log; exit 1; }
DB=$(find $O/svd -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 20 > $O/svd_kernels.txt 2>&1; rm -rf $O/svd
head -24 $O/svd_kernels.txt
