#!/bin/bash
# Round 5, final tree: the skewed configs[4] streams not yet measured on it
# (zipf-capped, fixed and CSR), with their full-shard parity.
set -o pipefail
O=${1:?outdir}
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O bench:--workload,tracker,$Q,--skew,zipf-capped \
  bench:--workload,tracker-csr,$Q,--skew,zipf-capped || exit 1
