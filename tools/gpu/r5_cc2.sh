#!/bin/bash
# Round 5: conf change placement pass with batched ID loads; composed
# wire -> tracker row; leader SQ counters.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_confchange.py || exit 1
bash tools/lab/ab_rows.sh 3 confchange tree base > $O/ab_confchange.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cc_prof -o run -- \
  python3 tools/bench_configs.py --only confchange --reps 10 --gpu-only > $O/cc_prof.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only wire-tracker --reps 10 --gpu-only \
  > $O/wire_tracker.json 2> $O/wire_tracker.err || { tail -5 $O/wire_tracker.err; exit 1; }
bash tools/gpu/r5_sq_ld.sh $O/sq > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
cat $O/ab_confchange.log $O/wire_tracker.json
