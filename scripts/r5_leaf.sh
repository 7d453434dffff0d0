#!/bin/bash
# Cholesky leaf kernel + small-tile GEMMs: phase probe, focused tests,
# isolated diagonal-block timings (new vs SLATE_POTRF_LEAF=0 SLATE_GEMM_SMALL=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_leaf; mkdir -p $O
bash scripts/r5_leafprobe.sh || exit 1
timeout -k 10 120 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider -k "potrf or gemm or trsm or posv or geqrf or cholqr" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== new"; timeout -k 10 120 python3 -u scripts/potrf_diag_probe.py 64,128,256,512,1024 || exit 1
echo "== old"; SLATE_POTRF_LEAF=0 SLATE_GEMM_SMALL=0 timeout -k 10 120 python3 -u scripts/potrf_diag_probe.py 512,1024 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p -o run -- python3 scripts/potrf_diag_probe.py 512 > /dev/null 2>&1 || exit 1
DB=$(find $O/p -name "*.db" | head -1); python3 scripts/panel_seq.py $DB --list > $O/seq.txt 2>&1; head -24 $O/seq.txt
