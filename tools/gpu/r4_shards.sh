#!/bin/bash
# Round 4: reserved-region shard count A/B (tools/lab/ab/s{1,2,4}.so, the
# tree = 8, base = round-3 bucketing) on both tracker ticks.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 bash tools/lab/ab_tracker.sh 2 tracker ${AB_LIBS} > $O/ab_tracker_shards.log 2>&1 || { cat $O/ab_tracker_shards.log; exit 1; }
cat $O/ab_tracker_shards.log
timeout -k 10 700 bash tools/lab/ab_tracker.sh 2 tracker-csr ${AB_LIBS} > $O/ab_tracker_csr_shards.log 2>&1 || { cat $O/ab_tracker_csr_shards.log; exit 1; }
cat $O/ab_tracker_csr_shards.log
