#!/bin/bash
# Round 4 end-of-round evidence: box info, the whole GPU suite, smoke, the
# driver's bench command, its kernel trace, and the headline kernel's
# FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains).
set -o pipefail
O=${1:?outdir}
P=--no-cpu-baseline,--no-parity,--no-others,--preroll-ms,0,--settle-ms,0,--steps,20,--warmup,5
bash tools/gpu/run.sh $O info tests smoke bench:--gpus,1,--steps,20,--warmup,5 \
  prof:--gpus,1,--steps,20,--warmup,5 pmc:FETCH_SIZE:$P pmc:WRITE_SIZE:$P
