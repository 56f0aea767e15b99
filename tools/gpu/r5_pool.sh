#!/bin/bash
# Round 5: the overflow pool (qb_bucket.h Pool) — the GPU suite, then the
# skewed streams on the new tree (compare profiles/r05/skew/*_before.json).
set -o pipefail
O=${1:?outdir}
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O tests \
  bench:--workload,tracker,$Q,--skew,sb10 bench:--workload,tracker,$Q,--skew,sb30 \
  bench:--workload,tracker-csr,$Q,--skew,sb10 bench:--workload,tracker-csr,$Q,--skew,sb30 \
  bench:--workload,tracker,$Q,--skew,zipf-capped bench:--workload,tracker,$Q,--skew,zipf
