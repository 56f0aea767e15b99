#!/bin/bash
# SQ counters of the conf-change row's kernels (k_cc_count, k_cc_move), one
# --pmc pass of 8 SQ counters.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/confchange_sq -o run -- \
  python3 tools/bench_configs.py --only confchange --gpu-only --reps 4 \
  > $O/confchange_sq.log 2>&1 || { echo "pmc failed"; tail -5 $O/confchange_sq.log; exit 1; }
python3 - $O <<'PY'
import csv, sys, re, statistics, glob
O = sys.argv[1]
f = glob.glob(f"{O}/confchange_sq/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").split("::")[-1]
    if k.startswith("k_cc"):
        per.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
for (k, c), v in sorted(per.items()):
    print(f"{k:28s} {c:18s} {statistics.median(v):16.0f}")
PY
