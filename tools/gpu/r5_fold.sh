#!/bin/bash
# Round 5: overflow pool + K4 fold + heavy-first apply — the GPU suite, the
# skewed streams, and the uniform tick / §8f rows A/B against the round-4
# build (tools/lab/ab/base.so, built from commit 6b05a42^).
set -o pipefail
O=${1:?outdir}
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O tests \
  bench:--workload,tracker,$Q,--skew,sb10 bench:--workload,tracker,$Q,--skew,sb30 \
  bench:--workload,tracker-csr,$Q,--skew,sb10 bench:--workload,tracker-csr,$Q,--skew,sb30 \
  bench:--workload,tracker,$Q,--skew,zipf bench:--workload,tracker-csr,$Q,--skew,zipf || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 3 tracker tree base > $O/ab_tracker.log 2>&1 || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker-csr tree base > $O/ab_tracker_csr.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 leader tree base > $O/ab_leader.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 readindex tree base > $O/ab_readindex.log 2>&1 || exit 1
cat $O/ab_*.log
