#!/bin/bash
# A/B of library builds on one §8f row of tools/bench_configs.py (GPU only):
# tools/lab/ab/<name>.so per name, "tree" = the in-tree build, alternating
# processes on one box.  Development tool.
#   ab_rows.sh <rounds> <row> name1 name2 ...
cd "$(dirname "$0")/../.."
rounds=$1; row=$2; shift 2
for i in $(seq $rounds); do
  for name in "$@"; do
    if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
    if timeout -k 10 150 python3 tools/bench_configs.py ${lp:+--lab-lib $lp} --only $row --reps 10 --gpu-only \
        > /tmp/abr_$name.json 2> /tmp/abr_$name.err; then
      echo "$name $(tail -1 /tmp/abr_$name.json)"
    else
      echo "$name FAILED rc=$?"; tail -5 /tmp/abr_$name.err
    fi
  done
done
