#!/bin/bash
# A/B previous commit (abprev/) vs working tree (new select kernel + PV ring), left-swap queue toggle
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "getrf or gesv or lu or qr or gels or tournament" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in "abprev" "." ".:SLATE_LU_LEFT_TRAIL=1"; do
    d=${v%%:*}; e=""; [ "$v" != "$d" ] && e=${v#*:}
    env $e timeout -k 10 400 python3 $d/bench.py --routines dgetrf --steps 1 --warmup 1 --extras cfg2_dpotrf_n32768_nb512 --extras-steps 1 --check no > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "== $v"; grep -E "step 1 timed" $O/b.log
  done
done
