#!/bin/bash
# Round 5: the driver's N = 8 command rehearsed on one GPU (8 spawned ranks,
# torch gloo collectives standing in for RCCL), wall time recorded.
set -o pipefail
O=${1:?outdir}
mkdir -p $O
s=$(date +%s)
timeout -k 10 1000 python -u bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 \
  > $O/bench_n8_gloo.json 2> $O/bench_n8_gloo.err
rc=$?
echo "rc=$rc wall_s=$(( $(date +%s) - s ))" | tee $O/bench_n8_gloo.wall
exit $rc
