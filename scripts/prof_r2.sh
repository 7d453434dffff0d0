#!/bin/bash
# round-2 evidence profiles: dgeqrf n=65536 kernel trace + GEMM timeline; zgemm kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2
N=65536 O=prof_r2/qr64k bash scripts/prof_qr.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r2/zgemm -o run -- bin/slate_tester gemm --type z --dim 16384 --nb 512 --target d --check n > gpurun_out/prof_r2/zgemm.log 2>&1 || exit 1
tail -3 gpurun_out/prof_r2/zgemm.log
DB=$(find gpurun_out/prof_r2/zgemm -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 10 > gpurun_out/prof_r2/zgemm_summary.txt; cat gpurun_out/prof_r2/zgemm_summary.txt
find gpurun_out/prof_r2 -name "*.db" -delete
