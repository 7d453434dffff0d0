#!/bin/bash
# PMC counters of the leaf kernels (bin/leaf_probe r = 960: potrf leaf + small trsm), one pass per group
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5_pmc; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- bin/leaf_probe 960 3 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM -d $O/p2 -o run --output-format csv -- bin/leaf_probe 960 3 > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
for p in p1 p2; do f=$(find $O/$p -name "*counter_collection.csv" | head -1); echo "== $p: $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", "?")).split("(")[0][-40:]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
done
