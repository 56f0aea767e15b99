#!/bin/bash
# Round 4: per-kernel traces of the §8f rows (leader, ReadIndex, wire, conf
# change) on the current tree.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for row in leader readindex wire confchange; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$row -o run -- \
    python3 tools/bench_configs.py --only $row --reps 10 --gpu-only > $O/$row.json 2> $O/$row.err \
    || { echo "prof $row failed"; tail -5 $O/$row.err; exit 1; }
done
for row in leader readindex wire confchange; do echo "== $row"; python3 tools/prof_summary.py $O/prof_$row/run_kernel_trace.csv; done > $O/summary.txt 2>&1 || true
echo ok
