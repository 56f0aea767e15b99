#!/bin/bash
# K4 fold threshold 512 -> 2048: tracker tests, then zipf-capped / zipf /
# uniform / sb30 ticks (with parity) and the zipf-capped + uniform A/B
# against the round-4 build.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O tests:test_gpu_tracker.py tests:test_gpu_tracker_csr.py \
  bench:--workload,tracker,$Q,--skew,zipf-capped bench:--workload,tracker-csr,$Q,--skew,zipf-capped \
  bench:--workload,tracker,$Q,--skew,zipf bench:--workload,tracker-csr,$Q,--skew,zipf \
  bench:--workload,tracker,$Q,--skew,sb30 bench:--workload,tracker-csr,$Q,--skew,sb30 || exit 1
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 2 tracker tree base > $O/ab_tracker_zc.log 2>&1 || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker tree base > $O/ab_tracker.log 2>&1 || exit 1
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 2 tracker-csr tree base > $O/ab_tracker_csr_zc.log 2>&1 || exit 1
cat $O/ab_*.log
