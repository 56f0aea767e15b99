#!/bin/bash
# Per-kernel rocprofv3 stats of one bench_configs config for several library
# builds (tools/lab/ab/<name>.so or "tree").  Development tool.
# Usage: prof_libs.sh <config> name1 name2 ...
set -e
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
cfg=$1; shift
for name in "$@"; do
  if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run \
    -- python3 tools/bench_configs.py ${lp:+--lab-lib $lp} --only $cfg --gpu-only --reps 20 > gpurun_out/prof_$name.log 2>&1
  f=$(find gpurun_out/prof_$name -name '*kernel_stats.csv' | head -1)
  echo "== $name"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:14]: print(f\"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f}\")"
done
