#!/bin/bash
# Round 4: SQ counters of the leader step's kernels, HEAD (head.so) vs the
# tree — one --pmc pass per library (8 SQ counters), k_ld_chunk_runs focus.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR"
for name in head tree; do
  if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/${name}_sq -o run -- \
    python3 tools/bench_configs.py ${lp:+--lab-lib $lp} --only leader --gpu-only --reps 4 \
    > $O/${name}_sq.log 2>&1 || { echo "pmc $name failed"; tail -5 $O/${name}_sq.log; exit 1; }
done
python3 - $O <<'PY'
import csv, sys, re, statistics, glob
O = sys.argv[1]
for name in ("head", "tree"):
    f = glob.glob(f"{O}/{name}_sq/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").split("::")[-1]
        if "chunk_runs" in k or "split" in k or "scatter" in k:
            per.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for (k, c), v in sorted(per.items()):
        print(name, f"{k:28s} {c:18s} {statistics.median(v):14.0f}")
PY
