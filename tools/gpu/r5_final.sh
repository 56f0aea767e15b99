#!/bin/bash
# Round 5 end-of-round evidence, part 1: box info, the whole GPU suite,
# smoke, the driver's bench command, its kernel trace, the headline kernel's
# FETCH_SIZE / WRITE_SIZE passes, and the tracker ticks' PMC passes
# (tools/gpu/pmc_tracker.sh).
set -o pipefail
O=${1:?outdir}
P=--no-cpu-baseline,--no-parity,--no-others,--preroll-ms,0,--settle-ms,0,--steps,20,--warmup,5
BENCH_TIMEOUT=600 bash tools/gpu/run.sh $O info tests smoke bench:--gpus,1,--steps,20,--warmup,5 \
  prof:--gpus,1,--steps,20,--warmup,5 pmc:FETCH_SIZE:$P pmc:WRITE_SIZE:$P || exit 1
bash tools/gpu/pmc_tracker.sh $O/pmc_tracker || exit 1
