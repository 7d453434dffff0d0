#!/bin/bash
# A/B the standalone GEMM harness binaries in tools_bin/ (old vs new kernel),
# then one PMC pass over the new one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-8192}
for b in ${BINS:-gemm_bench_old gemm_bench_new}; do
  echo "== $b"; timeout -k 10 120 ./tools_bin/$b $N || exit $?
done
if [ -n "$PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --stats -d gpurun_out/pmc -o pmc -- ./tools_bin/${PMC_BIN:-gemm_bench_new} $N > gpurun_out/pmc.log 2>&1 || exit $?
  echo pmc done
fi
