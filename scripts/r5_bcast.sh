#!/bin/bash
# SLATE_BCAST variants: correctness on the shared-GPU RCCL rig + kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_bcast; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist.py -k "bcast_modes" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "variants_all_types" > $O/pytest_var.log 2>&1 || { tail -30 $O/pytest_var.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_var.log
for MODE in rccl sendrecv tree; do
  SLATE_BCAST=$MODE RANK_LOGDIR=$O/ranks_$MODE RANK_TIMEOUT=200 timeout -k 10 240 python3 scripts/rccl_multi.py 4 --cmd rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_$MODE -o r%pid% -- bin/slate_tester potrf --type d --dim 2048 --nb 256 --grid 2x2 --target d > $O/run_$MODE.log 2>&1 || { tail -20 $O/run_$MODE.log; exit 1; }
  grep -c "pass" $O/run_$MODE.log
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_examples.py tests/test_gpu.py -k "inproc_transparent" > $O/pytest_inproc.log 2>&1 || { tail -40 $O/pytest_inproc.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_inproc.log
