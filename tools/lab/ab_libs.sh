#!/bin/bash
# A/B of library builds: tools/lab/ab/<name>.so for each name given, plus the
# in-tree build ("tree"), alternating processes on one box, `rounds` rounds.
# Usage: ab_libs.sh "<configs>" rounds name1 name2 ...   Development tool.
set -e
cd "$(dirname "$0")/../.."
cfg=$1; rounds=$2; shift 2
for i in $(seq $rounds); do
  for name in "$@"; do
    if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
    timeout -k 10 150 python tools/bench_configs.py ${lp:+--lab-lib $lp} --only $cfg --gpu-only --reps 20 2>/dev/null \
      | python -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$name', d['config'][:40], 'us', round(d['per_launch_us'],1), 'frac', round(d.get('frac_hbm_peak',0),3), flush=True)"
  done
done
