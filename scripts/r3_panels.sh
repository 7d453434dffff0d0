#!/bin/bash
# round-3 panel work: tournament v2 + QR panel explicit V: tests, isolated panels, benches, trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/panels; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "getrf or permute or trsm or gesv or lu or qr or gels or unmqr or larfb" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for mode in 0 1; do
  for m in 2048 32768; do
    SLATE_TSLU_WG=$mode PANELS=tournament timeout -k 10 120 python3 scripts/bench_panel.py $m 1024 2>&1 | grep -v "^W2026\|amdgpu.ids" | sed "s/^/wg=$mode /" >> $O/panel.txt || exit 1
  done
done
for m in 2048 32768; do
  PANELS=geqrf timeout -k 10 120 python3 scripts/bench_panel.py $m 512 2>&1 | grep -v "^W2026\|amdgpu.ids" >> $O/panel.txt || exit 1
done
cat $O/panel.txt
for v in "" "SLATE_LU_LEFT_TRAIL=1" "SLATE_TSLU_WG=1"; do
  env $v timeout -k 10 300 python3 bench.py --routines dgetrf --steps 1 --warmup 1 --extras none > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  echo "== $v"; grep -E "timed|error" $O/bench.log
done
timeout -k 10 300 python3 bench.py --routines dgeqrf --steps 1 --warmup 1 --extras none > $O/bench_qr.log 2>&1 || { tail -20 $O/bench_qr.log; exit 1; }
grep -E "timed|error" $O/bench_qr.log
