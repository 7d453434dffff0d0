#!/bin/bash
# PMC counters of the TSQR node kernel on the isolated QR panel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_panel; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --kernel-include-regex "qr_node_kernel" -d $O -o p -- python3 scripts/bench_panel.py 65536 512 > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
DB=$(find $O -name "*.db" | head -1)
python3 scripts/pmc_summary.py $DB qr_node | head -60
rm -f $DB
