#!/bin/bash
# Round 6: Cholesky on 8 x 1 -- nb check in the model and the 8-rank rig residuals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_potrf8x1; mkdir -p $O
GRIDS="8x1" NBS="768 1024" ROUT=chol scripts/r6_sweep24.sh | sed -E 's/steps whose.*CU-free comm [0-9.]+\) //'
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 600 python3 -u bench.py --gpus 8 --dim 16384 --routines dpotrf --steps 1 --warmup 0 --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 > $O/b8.txt 2> $O/b8.err || { tail -20 $O/b8.err; exit 1; }
grep -E "backward" $O/b8.err
tail -1 $O/b8.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: (v['grid'], v['nb']) for k, v in d['routines'].items()})"
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 400 python3 -u bench.py --gpus 4 --dim 16384 --routines dpotrf --steps 1 --warmup 0 --extras none > $O/b4.txt 2> $O/b4.err || { tail -20 $O/b4.err; exit 1; }
grep -E "backward" $O/b4.err
