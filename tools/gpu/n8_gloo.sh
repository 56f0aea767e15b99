#!/bin/bash
# The driver's N = 8 command rehearsed on one GPU: 8 ranks spawned by
# bench.py, torch gloo collectives standing in for RCCL; wall time recorded.
#   tools/gpu/n8_gloo.sh OUTDIR
set -o pipefail
O=${1:?outdir}
mkdir -p $O
s=$(date +%s)
timeout -k 10 1000 python -u bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 \
  > $O/bench_n8_gloo.json 2> $O/bench_n8_gloo.err
rc=$?
echo "rc=$rc wall_s=$(( $(date +%s) - s ))" | tee $O/bench_n8_gloo.wall
exit $rc
