#!/bin/bash
# rocprofv3 kernel trace of dgeqrf (n from $N, default 32768) + kernel summary + GEMM timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
N=${N:-32768}; O=${O:-prof_qr}
mkdir -p gpurun_out/$O
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/$O -o run -- python3 bench.py --routines ${R:-dgeqrf} --steps 1 --warmup 0 --dim $N --extras none --check no ${BENCH_ARGS:-} > gpurun_out/$O/bench.log 2>&1 || exit $?
grep timed gpurun_out/$O/bench.log
DB=$(find gpurun_out/$O -name "*.db" | head -1)
python3 scripts/prof_summary.py $DB 30 > gpurun_out/$O/summary.txt && python3 scripts/timeline.py $DB >> gpurun_out/$O/summary.txt
cat gpurun_out/$O/summary.txt
rm -f $DB
