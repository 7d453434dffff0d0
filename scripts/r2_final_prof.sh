#!/bin/bash
# End-of-round kernel traces (summary + GEMM timeline) of the factorizations at
# n=65536 and the config-2 dpotrf, with the round-2 panel changes in place.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in dpotrf dgetrf dgeqrf; do
  R=$r N=65536 O=final_prof/$r bash scripts/prof_qr.sh > /dev/null || { echo "$r prof failed"; exit 1; }
  head -1 gpurun_out/final_prof/$r/summary.txt; grep -e "gemm-covered" gpurun_out/final_prof/$r/summary.txt | head -1
done
R=dpotrf N=32768 BENCH_ARGS="--nb 512" O=final_prof/dpotrf_cfg2 bash scripts/prof_qr.sh > /dev/null || { echo "cfg2 prof failed"; exit 1; }
head -1 gpurun_out/final_prof/dpotrf_cfg2/summary.txt; grep -e "gemm-covered" gpurun_out/final_prof/dpotrf_cfg2/summary.txt | head -1
