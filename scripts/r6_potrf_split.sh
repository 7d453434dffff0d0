#!/bin/bash
# Round 6: p x q Cholesky with the transposed tiles in two all-gathers (lookahead columns first):
# rig tests (staircase path over RCCL), then the 4 x 2 model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_potrf_split; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -m gpu -k "potrf or 2x4 or bcast_modes or no_fast or multirank" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep -cE "PASSED" $O/pytest.txt; tail -1 $O/pytest.txt
SLATE_PANEL_CUS=32 timeout -k 10 300 python3 -u scripts/critpath.py --p 4 --q 2 --nb 512 --every 16 --reps 2 --routines chol > $O/chol.txt 2>&1 || { tail -5 $O/chol.txt; exit 1; }
grep -E "sampled sums|CU-free messages" $O/chol.txt
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 500 python3 -u bench.py --gpus 8 --dim 16384 --routines dpotrf --steps 1 --warmup 0 --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 > $O/b8.txt 2> $O/b8.err || { tail -20 $O/b8.err; exit 1; }
grep -E "backward" $O/b8.err
