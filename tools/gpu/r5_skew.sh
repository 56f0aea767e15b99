#!/bin/bash
# Round 5: the GPU suite, the driver's command (generator-based bench), and the
# configs[4] skewed-batch streams next to the uniform tick (VERDICT r4 Next 2).
set -o pipefail
O=${1:?outdir}
Q=--no-cpu-baseline
bash tools/gpu/run.sh $O info tests bench:--gpus,1,--steps,20,--warmup,5 \
  bench:--workload,tracker,$Q,--skew,none bench:--workload,tracker,$Q,--skew,zipf-capped \
  bench:--workload,tracker,$Q,--skew,sb10 bench:--workload,tracker,$Q,--skew,sb30 \
  bench:--workload,tracker-csr,$Q,--skew,none bench:--workload,tracker-csr,$Q,--skew,zipf-capped \
  bench:--workload,tracker-csr,$Q,--skew,sb10 bench:--workload,tracker-csr,$Q,--skew,sb30 \
  bench:--workload,tracker,$Q,--skew,zipf
