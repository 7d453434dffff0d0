#!/bin/bash
# A/B two standalone GEMM harness builds: correctness + 8192 timings + a big NN/NT/TN run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in ${BINS:-gemm_bench_kxl0 gemm_bench_kxl1}; do
  echo "== $b"; timeout -k 10 120 ./tools_bin/$b 8192 | grep -v "^check" || exit $?
  timeout -k 10 120 ./tools_bin/$b ${BIG:-32768 16384 0 1} | tail -3 || exit $?
done
