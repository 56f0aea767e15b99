#!/bin/bash
# Escape column for escape-dense K3 tiles only: tracker tests, per-kernel
# trace, A/B against the build before (r5h), the composed row (all-escape).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_tracker.py tests:test_gpu_tracker_csr.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tree -o run -- \
  python3 bench.py --workload tracker --no-cpu-baseline --no-parity --steps 20 --warmup 5 \
  > $O/tree.json 2> $O/tree.err || { tail -5 $O/tree.err; exit 1; }
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 3 tracker tree r5h > $O/ab_tracker.log 2>&1 || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker-csr tree r5h > $O/ab_tracker_csr.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only wire-tracker --reps 10 --gpu-only \
  > $O/wire_tracker.json 2> $O/wire_tracker.err || { tail -5 $O/wire_tracker.err; exit 1; }
cut -d, -f1-4 $O/tree/run_kernel_stats.csv | head -4
cat $O/ab_tracker.log $O/ab_tracker_csr.log $O/wire_tracker.json
