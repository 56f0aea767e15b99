#!/bin/bash
# Which part of the escape column costs the uniform tick: tree vs foot (the
# column's carve only; round-4 escape path) vs r5h (before the column).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for name in tree foot r5h; do
  if [ $name = tree ]; then lp=""; else lp="--lab-lib $PWD/tools/lab/ab/$name.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 bench.py $lp --workload tracker --no-cpu-baseline --no-parity --steps 20 --warmup 5 \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
done
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker tree foot r5h > $O/ab_tracker.log 2>&1 || exit 1
for name in tree foot r5h; do echo $name; cut -d, -f1-4 $O/$name/run_kernel_stats.csv | head -4; done
cat $O/ab_tracker.log
