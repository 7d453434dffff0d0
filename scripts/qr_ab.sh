cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then export SLATE_QR_PANEL=old; else unset SLATE_QR_PANEL; fi
  echo "== $v"; timeout -k 10 120 python scripts/bench_panel.py 65536 512 2>&1 | grep geqrf || exit 1
done
mkdir -p gpurun_out/pq
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pq -o run -- python3 bench.py --routines dgeqrf --dim 32768 --steps 1 --warmup 0 > gpurun_out/pq/log 2>&1 || exit 1
echo prof ok
