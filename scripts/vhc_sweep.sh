#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in "512 32768 32768" "512 20000 44000" "512 8192 57344" "512 48000 16000"; do
  timeout -k 10 120 ./tools_bin/gemm_bench vhc $a 3 >> gpurun_out/vhc.txt 2>&1 || exit $?
done
cat gpurun_out/vhc.txt
