#!/bin/bash
# Round 6: peer broadcast with wait_ipc (query / stream wait / host poll): rig tests + 2-rank bench with extras.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_peer2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_dist.py -k "bcast_modes" > $O/pytest_bcast.txt 2>&1 || { tail -40 $O/pytest_bcast.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_bcast.txt | tail -14
SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 500 python3 -u bench.py --gpus 2 --dim 16384 --steps 1 --warmup 1 > $O/b2.txt 2> $O/b2.err || { tail -40 $O/b2.err; exit 1; }
grep -v amdgpu $O/b2.err | grep -c pass
tail -1 $O/b2.txt | cut -c1-300
for mk in 2048 1000 2048 1000; do SLATE_GEMM_PACK_A_MINK=$mk timeout -k 10 120 python3 -u scripts/r6_gemm_k.py >> $O/gemm_k.txt 2>&1 || { tail -5 $O/gemm_k.txt; exit 1; }; done
grep mink $O/gemm_k.txt
