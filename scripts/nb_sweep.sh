#!/bin/bash
# nb / lookahead sweep of the headline routines at n=65536 (1 GPU), one process per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
run() {  # name routine args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --steps 1 --warmup 1 "$@" > gpurun_out/sweep/$name.log 2>&1 || { echo "$name FAILED rc=$?"; tail -5 gpurun_out/sweep/$name.log; exit 1; }
  echo "$name: $(grep -h 'step 1 timed' gpurun_out/sweep/$name.log | tr '\n' ' ')"
}
run getrf_512      --routines dgetrf --nb 512
run getrf_768      --routines dgetrf --nb 768
run getrf_1024     --routines dgetrf --nb 1024
run getrf_512_la2  --routines dgetrf --nb 512 --lookahead 2
run potrf_768      --routines dpotrf --nb 768
run potrf_1024     --routines dpotrf --nb 1024
run geqrf_512_la2  --routines dgeqrf --nb 512 --lookahead 2
run geqrf_384      --routines dgeqrf --nb 384
