#!/bin/bash
# Per-kernel trace of the uniform fixed tracker tick: tree vs lab builds
# (tools/lab/ab/<name>.so), then alternating A/B of the fixed and CSR ticks,
# and the composed wire -> tracker row.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_tracker.py tests:test_gpu_tracker_csr.py || exit 1
for name in tree r5h; do
  if [ $name = tree ]; then lp=""; else lp="--lab-lib $PWD/tools/lab/ab/$name.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 bench.py $lp --workload tracker --no-cpu-baseline --no-parity --steps 20 --warmup 5 \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
done
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker tree r5h base > $O/ab_tracker.log 2>&1 || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker-csr tree r5h base > $O/ab_tracker_csr.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only wire-tracker --reps 10 --gpu-only \
  > $O/wire_tracker.json 2> $O/wire_tracker.err || { tail -5 $O/wire_tracker.err; exit 1; }
for name in tree r5h; do echo $name; cut -d, -f1-4 $O/$name/run_kernel_stats.csv | head -5; done
cat $O/ab_tracker.log $O/ab_tracker_csr.log $O/wire_tracker.json
