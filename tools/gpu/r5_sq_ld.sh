#!/bin/bash
# Round 5: SQ counters of the leader step's kernels (the leader and ReadIndex
# rows of tools/bench_configs.py), one --pmc pass per row (8 SQ counters).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
for row in leader readindex; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/${row}_sq -o run -- \
    python3 tools/bench_configs.py --only $row --gpu-only --reps 4 \
    > $O/${row}_sq.log 2>&1 || { echo "pmc $row failed"; tail -5 $O/${row}_sq.log; exit 1; }
done
python3 - $O <<'PY'
import csv, sys, re, statistics, glob
O = sys.argv[1]
for row in ("leader", "readindex"):
    f = glob.glob(f"{O}/{row}_sq/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").split("::")[-1]
        if k.startswith("k_ld") or "split" in k or "scatter" in k:
            per.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for (k, c), v in sorted(per.items()):
        print(row, f"{k:28s} {c:18s} {statistics.median(v):16.0f}")
PY
