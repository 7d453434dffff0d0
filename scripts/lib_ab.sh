#!/bin/bash
# A/B the framework against alternative builds of libslate_amd.so placed in
# tools_bin/lib_<name>/ (LD_LIBRARY_PATH beats the extension's RUNPATH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${ARGS:---routines dpotrf,dgetrf,dgeqrf --dim 32768 --steps 1 --warmup 1}
for v in ${LIBS:-old a h}; do
  LD_LIBRARY_PATH=$PWD/tools_bin/lib_$v timeout -k 10 ${T:-300} python bench.py $ARGS > gpurun_out/lib_$v.log 2>&1 || exit 1
  echo "== $v"; grep timed gpurun_out/lib_$v.log
done
