#!/bin/bash
# Round 5 end-of-round evidence, part 2: per-kernel time and HBM traffic of
# the §8f rows and the composed row (tools/gpu/rows.sh), then the driver's
# N = 8 command rehearsed on one GPU with gloo (tools/gpu/r5_n8.sh).
set -o pipefail
O=${1:?outdir}
bash tools/gpu/rows.sh $O/rows "leader readindex wire confchange wire-tracker" || exit 1
bash tools/gpu/r5_n8.sh $O/multi || exit 1
