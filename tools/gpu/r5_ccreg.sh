#!/bin/bash
# Conf change count pass with its kSmall table in registers: conf change
# tests, A/B against the committed build (hd), kernel trace.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_confchange.py || exit 1
bash tools/lab/ab_rows.sh 3 confchange tree hd > $O/ab_confchange.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cc_prof -o run -- \
  python3 tools/bench_configs.py --only confchange --reps 10 --gpu-only > $O/cc_prof.log 2>&1 || exit 1
cut -d, -f1-4 $O/cc_prof/run_kernel_stats.csv | head -5
cat $O/ab_confchange.log
