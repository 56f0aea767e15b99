#!/bin/bash
# Round 5 end-of-round evidence on the final tree (K4 fold threshold 2048):
# part 1 (tools/gpu/r5_final.sh) and the sb10 skewed ticks.
set -o pipefail
O=${1:?outdir}
bash tools/gpu/r5_final.sh $O || exit 1
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O/skew bench:--workload,tracker,$Q,--skew,sb10 \
  bench:--workload,tracker-csr,$Q,--skew,sb10 || exit 1
