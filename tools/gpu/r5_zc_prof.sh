#!/bin/bash
# Per-kernel trace of the zipf-capped fixed tick: the final tree vs the
# round-4 build.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for name in tree base; do
  if [ $name = tree ]; then lp=""; else lp="--lab-lib $PWD/tools/lab/ab/$name.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 bench.py $lp --workload tracker --no-cpu-baseline --no-parity --skew zipf-capped --steps 20 --warmup 5 \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
done
for name in tree base; do echo $name; cut -d, -f1-4 $O/$name/run_kernel_stats.csv | head -6; done
