#!/bin/bash
# Round 6: the per-world grid / nb defaults on the shared-GPU rig (ranks on one
# MI355X, RCCL socket transport): every routine's residual must pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_grids; mkdir -p $O
for nd in "2 16384" "4 16384" "8 8192"; do
  set -- $nd
  SLATE_BENCH_FAKE_HOSTS=1 timeout -k 10 500 python3 -u bench.py --gpus $1 --dim $2 --steps 1 --warmup 1 --extras none > $O/b$1.txt 2> $O/b$1.err || { tail -30 $O/b$1.err; exit 1; }
  echo "N=$1: $(grep -E 'backward' $O/b$1.err | tr '\n' ' ')"
  tail -1 $O/b$1.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: (v['grid'], v['nb']) for k, v in d['routines'].items()}, d['config']['model'])"
done
