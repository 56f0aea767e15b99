#!/bin/bash
# Round 4: FETCH_SIZE / WRITE_SIZE of the leader step's kernels, HEAD (head.so)
# vs the tree (separate --pmc passes, one counter group each).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for name in head tree; do
  if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o run -- \
      python3 tools/bench_configs.py ${lp:+--lab-lib $lp} --only leader --gpu-only --reps 4 \
      > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, sys, re, statistics, glob
O = sys.argv[1]
for name in ("head", "tree"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{O}/{name}_{c}/**/*counter_collection.csv", recursive=True)[0]
        per = {}
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").split("::")[-1]
            if "k_ld" in k or "k_bk" in k:
                per.setdefault(k, []).append(float(r["Counter_Value"]))
        for k, v in sorted(per.items()):
            mult = 2 if c == "FETCH_SIZE" else 1
            print(name, c, f"{k:28s} MB {statistics.median(v) * mult / 1024:9.1f}")
PY
