#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/nb2048; mkdir -p $O
for e in "" "SLATE_UPDATE_NT=0" "SLATE_TSLU_WG=1"; do
  echo "== $e"
  env $e timeout -k 10 200 bin/slate_tester getrf --type d --dim 4096,6000 --nb 2048,1536,1280,1024 --target d --check y > $O/t.log 2>&1; grep -E "getrf" $O/t.log
done
timeout -k 10 200 bin/slate_tester getrf --type d --dim 4096 --nb 2048 --target d --check y --lookahead 0 > $O/t.log 2>&1; echo "== la0"; grep getrf $O/t.log
