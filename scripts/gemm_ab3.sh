#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in ${BINS}; do
  echo "== $b"; timeout -k 10 120 ./tools_bin/$b 8192 | grep -v "^check" || exit $?
  timeout -k 10 120 ./tools_bin/$b ${BIG:-16384 16384 0 2} | tail -3 || exit $?
  timeout -k 10 120 ./tools_bin/$b 32768 512 0 5 | tail -3 || exit $?
done
