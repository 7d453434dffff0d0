#!/bin/bash
# Interleaved A/B/C... of GEMM harness builds (two rounds) on big shapes only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
for b in ${BINS}; do
  out=$(timeout -k 10 120 ./tools_bin/$b 16384 16384 0 2 | tail -3; timeout -k 10 120 ./tools_bin/$b 32768 512 0 5 | tail -3) || exit 1
  echo "$b r$round: $(echo "$out" | awk '{print $2"/"$4"="$(NF-1)}' | tr '\n' ' ')"
done
done
