#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in "65536 512 0 3" "65536 1024 0 3" "32768 512 0 5" "16384 512 0 10" "65536 256 0 3"; do
  timeout -k 10 120 ./tools_bin/${BIN:-gemm_bench_rot1} $a | tail -3 || exit $?
done
