#!/bin/bash
# A/B of the leader step: baseline build (tools/lab/ab/libquorumbatch_base.so)
# vs the in-tree build, alternating processes on one box.  Development tool.
set -e
cd "$(dirname "$0")/../.."
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_configs.py --lab-lib $PWD/tools/lab/ab/libquorumbatch_base.so --only ${1:-leader} --gpu-only --reps 20 2>/dev/null | sed 's/^/base /'
  timeout -k 10 120 python tools/bench_configs.py --only ${1:-leader} --gpu-only --reps 20 2>/dev/null | sed 's/^/new  /'
done
