#!/bin/bash
# K4 fold threshold 1024: zipf-capped / zipf ticks (with parity) and the
# zipf-capped A/B against the round-4 build.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O tests:test_gpu_tracker.py::test_step_hot_groups_fold_in_k4 \
  tests:test_gpu_tracker_csr.py::test_csr_step_hot_groups_fold_in_k4 \
  bench:--workload,tracker,$Q,--skew,zipf-capped bench:--workload,tracker-csr,$Q,--skew,zipf-capped \
  bench:--workload,tracker,$Q,--skew,zipf bench:--workload,tracker-csr,$Q,--skew,zipf || exit 1
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 2 tracker tree base > $O/ab_tracker_zc.log 2>&1 || exit 1
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 2 tracker-csr tree base > $O/ab_tracker_csr_zc.log 2>&1 || exit 1
cat $O/ab_*.log
