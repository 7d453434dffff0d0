#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for M in 32768 1024; do
  timeout -k 5 60 bin/tslu_probe $M 20 512 || exit 1
done
