#!/bin/bash
# potrf leaf kernel phase timings (bin/leaf_probe, built with -DLEAF_PROBE)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 0 960; do
  timeout -k 5 60 bin/leaf_probe $r 20 || exit 1
done
