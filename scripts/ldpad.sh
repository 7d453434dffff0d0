cd "${GRAFT_REPO_ROOT}"
for args in "32768 32768 0" "32768 32768 64" "65536 8192 0" "65536 8192 64" "65536 8192 128"; do
  timeout -k 10 120 ./tools_bin/gemm_bench_rot1 $args 1 || exit $?
done
