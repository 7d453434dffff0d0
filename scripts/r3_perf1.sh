#!/bin/bash
# Round 3 perf probe: eig/svd stage-2 kernels, standalone sgemm, dgemm pack-A
# A/B, dgesv_mixed, and a dgetrf kernel trace at n=65536.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/perf1
O=gpurun_out/perf1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "svd or heev or eig or bdsqr" > $O/pytest_eig.log 2>&1 || { tail -30 $O/pytest_eig.log; exit 1; }
tail -1 $O/pytest_eig.log
timeout -k 10 300 python -u scripts/eig_prof.py 8192 256 d heev,svd > $O/eig_prof.log 2>&1 || { tail -20 $O/eig_prof.log; exit 1; }
grep -E "^(heev|svd)|bdsqr|tb2bd|hb2st|unmtr_hb2st_blocked|stedc_dist" $O/eig_prof.log
timeout -k 10 300 bin/slate_tester gemm --type s,d --dim 16384,65536x65536x1024 --nb 512 --target d --check n --repeat 2 > $O/sgemm.log 2>&1 || { tail -20 $O/sgemm.log; exit 1; }
grep gemm $O/sgemm.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/sgemm_prof -o run -- bin/slate_tester gemm --type s --dim 16384 --nb 512 --target d --check n > $O/sgemm_prof.log 2>&1 || { tail -20 $O/sgemm_prof.log; exit 1; }
find $O/sgemm_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} head -5 {}
for v in default unsliced; do
  if [ $v = unsliced ]; then export SLATE_GEMM_PACK_BYTES=1000000000000; fi
  timeout -k 10 200 python bench.py --routines dgemm --steps 1 --warmup 1 --extras none --check no > $O/dgemm_$v.log 2>&1 || { tail -20 $O/dgemm_$v.log; exit 1; }
  echo "== dgemm $v"; grep timed $O/dgemm_$v.log
done
unset SLATE_GEMM_PACK_BYTES
timeout -k 10 300 bin/slate_tester gesv_mixed --type d --dim 65536 --nb 1024 --target d --check y > $O/gesv_mixed.log 2>&1 || { tail -20 $O/gesv_mixed.log; exit 1; }
grep gesv_mixed $O/gesv_mixed.log
R=dgetrf N=65536 BENCH_ARGS="--method-lu tntpiv" O=perf1/prof_getrf bash scripts/prof_qr.sh > /dev/null || { echo "getrf prof failed"; exit 1; }
head -12 $O/prof_getrf/summary.txt; grep -A14 "gemm-covered" $O/prof_getrf/summary.txt | head -16
