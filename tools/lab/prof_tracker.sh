#!/bin/bash
# Per-kernel rocprofv3 stats of the tracker bench workloads for several
# library builds (tools/lab/ab/<name>.so or "tree").  Development tool.
# Usage: prof_tracker.sh <workload> name1 name2 ...
set -e
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
wl=$1; shift
for name in "$@"; do
  if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_$name -o run \
    -- python3 bench.py ${lp:+--lab-lib $lp} --workload $wl --no-cpu-baseline --steps 20 --warmup 5 \
    > gpurun_out/prof_${wl}_$name.log 2>&1
  f=$(find gpurun_out/prof_${wl}_$name -name '*kernel_stats.csv' | head -1)
  echo "== $name"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows:
    if r['Name'].startswith('qb::') or r['Name'].startswith('void qb::'):
        print(f\"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f}\")"
done
