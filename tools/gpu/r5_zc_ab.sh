#!/bin/bash
# zipf-capped configs[4] streams: the final tree against the round-4 build
# (tools/lab/ab/base.so), alternating processes on one box.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 3 tracker tree base > $O/ab_tracker_zc.log 2>&1 || exit 1
AB_ARGS="--no-parity --skew zipf-capped" bash tools/lab/ab_tracker.sh 2 tracker-csr tree base > $O/ab_tracker_csr_zc.log 2>&1 || exit 1
cat $O/ab_tracker_zc.log $O/ab_tracker_csr_zc.log
