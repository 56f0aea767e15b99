#!/bin/bash
# The leader GPU suite after bounding the meta word's counts (incl. the new
# bounded-meta test).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_leader.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests_leader.log 2>&1 || { tail -30 $O/gpu_tests_leader.log; exit 1; }
tail -2 $O/gpu_tests_leader.log
