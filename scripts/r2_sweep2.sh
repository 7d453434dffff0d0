#!/bin/bash
# Round-2 sweep after the TSQR panel / split-K changes: dgeqrf nb and lookahead,
# dpotrf at the BASELINE config-2 size (n=32768, nb=512) with lookahead 1-3,
# and the partial-pivoting (ppiv) LU at n=65536.  One process per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep2
run() {  # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --extras none --check no "$@" > gpurun_out/sweep2/$name.log 2>&1 || { echo "$name FAILED rc=$?"; tail -5 gpurun_out/sweep2/$name.log; exit 1; }
  echo "$name: $(grep -h 'step 1 timed' gpurun_out/sweep2/$name.log | tr '\n' ' ')"
}
run potrf32k_512_la1 --routines dpotrf --n 32768 --nb 512 --lookahead 1
run potrf32k_512_la2 --routines dpotrf --n 32768 --nb 512 --lookahead 2
run potrf32k_512_la3 --routines dpotrf --n 32768 --nb 512 --lookahead 3
run geqrf_640        --routines dgeqrf --nb 640
run geqrf_768        --routines dgeqrf --nb 768
run geqrf_512_la2    --routines dgeqrf --nb 512 --lookahead 2
run getrf_ppiv_1024  --routines dgetrf --nb 1024 --method-lu ppiv
run potrf_1024_la2   --routines dpotrf --nb 1024 --lookahead 2
