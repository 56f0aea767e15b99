#!/bin/bash
# Leader grouping fused into the step (k_ld_step_fused, sparse batches):
# leader + wire tests, per-kernel trace of the leader row, A/B of leader /
# ReadIndex against the committed build (hd).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_leader.py tests:test_gpu_wire.py || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/leader_trace -o run -- \
  python3 tools/bench_configs.py --only leader --reps 10 --gpu-only > $O/leader_trace.jsonl 2> $O/leader_trace.err || exit 1
bash tools/lab/ab_rows.sh 3 leader tree hd > $O/ab_leader.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 readindex tree hd > $O/ab_readindex.log 2>&1 || exit 1
cut -d, -f1-4 $O/leader_trace/run_kernel_stats.csv | head -12
cat $O/ab_leader.log $O/ab_readindex.log
