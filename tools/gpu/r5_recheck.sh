#!/bin/bash
# Round 5 closing re-check on the committed tree (library rebuilt by build()
# after a warning fix that leaves the device code unchanged): box info, the
# whole GPU suite, smoke, the driver's bench command.
set -o pipefail
O=${1:?outdir}
BENCH_TIMEOUT=600 bash tools/gpu/run.sh $O info tests smoke bench:--gpus,1,--steps,20,--warmup,5 || exit 1
