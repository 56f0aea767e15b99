#!/bin/bash
# Round 4: reserved-region capacity sized from the fullest super-bucket in
# 256-record granules — the tracker GPU tests (incl. the 128M tick), then
# alternating-process A/B against the previous cap (tools/lab/ab/s8.so).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py \
  tests/test_gpu_capacity.py::test_fixed_tracker_tick_128m_groups_one_device -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tracker_tests.log 2>&1 \
  || { echo "tracker tests failed"; tail -40 $O/tracker_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/tracker_tests.log)"
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker s8 tree > $O/ab_tracker.log 2>&1 || { cat $O/ab_tracker.log; exit 1; }
cat $O/ab_tracker.log
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker-csr s8 tree > $O/ab_tracker_csr.log 2>&1 || { cat $O/ab_tracker_csr.log; exit 1; }
cat $O/ab_tracker_csr.log
