#!/bin/bash
# Reserved panel CUs (SLATE_PANEL_CUS) for the config-2 dpotrf (n=32768, nb=512)
# and the n=65536 factorizations, one process per setting on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cus
for c in 0 4 8 16 0; do
  SLATE_PANEL_CUS=$c timeout -k 10 120 python bench.py --routines dpotrf --n 32768 --nb 512 --steps 3 --warmup 1 --extras none --check no > gpurun_out/cus/p32_$c.log 2>&1 || { echo "cus=$c FAILED"; tail -5 gpurun_out/cus/p32_$c.log; exit 1; }
  echo "potrf32k cus=$c: $(grep -h 'timed' gpurun_out/cus/p32_$c.log | tr '\n' ' ')"
done
for c in 8 0; do
  SLATE_PANEL_CUS=$c timeout -k 10 200 python bench.py --routines dpotrf,dgetrf,dgeqrf --steps 1 --warmup 1 --extras none --check no > gpurun_out/cus/big_$c.log 2>&1 || { echo "cus=$c FAILED"; tail -5 gpurun_out/cus/big_$c.log; exit 1; }
  echo "64k cus=$c: $(grep -h 'step 1 timed' gpurun_out/cus/big_$c.log | tr '\n' ' ')"
done
