#!/bin/bash
# A/B of lab builds (tools/lab/ab/<name>.so, "tree" = in-tree) on the
# tracker workloads.  Usage: tools/gpu/ab.sh OUT ROUNDS "names" ["csr names"]
set -o pipefail
O=${1:?out}; R=$2; mkdir -p $O
bash tools/lab/ab_tracker.sh $R tracker $3 > $O/ab_tracker.log 2>&1 || exit 1
cat $O/ab_tracker.log
if [ -n "$4" ]; then
  bash tools/lab/ab_tracker.sh $R tracker-csr $4 > $O/ab_tracker_csr.log 2>&1 || exit 1
  cat $O/ab_tracker_csr.log
fi
