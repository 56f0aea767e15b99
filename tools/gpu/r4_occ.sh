#!/bin/bash
# Round 4: k_ld_step at 5 waves per SIMD (1280 staged slots, waves_per_eu(5):
# 96 VGPRs with 15 spilled) vs the tree (4 waves) on the leader / ReadIndex rows.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for row in leader readindex; do
  timeout -k 10 600 bash tools/lab/ab_rows.sh 3 $row tree occ5 > $O/ab_$row.log 2>&1 || { echo "ab $row failed"; cat $O/ab_$row.log; exit 1; }
done
python3 - $O <<'PY'
import json, sys
for f in ("ab_leader.log", "ab_readindex.log"):
    for line in open(f"{sys.argv[1]}/{f}"):
        name, _, js = line.partition(" ")
        try:
            d = json.loads(js)
            print(f, name, round(d["per_launch_us"], 1), round(d.get("ordered_us", 0), 1))
        except Exception:
            print(f, line.strip())
PY
