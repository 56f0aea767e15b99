#!/bin/bash
# Round 4: the tracker steps with reserved regions (no K1 histogram, scan or
# part table) — the tracker GPU tests, then alternating-process A/B against
# the previous build (tools/lab/ab/base.so) and a kernel trace of each tick.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py \
  tests/test_gpu_capacity.py::test_fixed_tracker_tick_128m_groups_one_device -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tracker_tests.log 2>&1 \
  || { echo "tracker tests failed"; tail -40 $O/tracker_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/tracker_tests.log)"
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker base tree > $O/ab_tracker.log 2>&1 || { cat $O/ab_tracker.log; exit 1; }
cat $O/ab_tracker.log
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker-csr base tree > $O/ab_tracker_csr.log 2>&1 || { cat $O/ab_tracker_csr.log; exit 1; }
cat $O/ab_tracker_csr.log
for wl in tracker tracker-csr; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 bench.py --workload $wl --no-cpu-baseline --no-parity > $O/prof_$wl.json 2> $O/prof_$wl.err \
    || { echo "prof $wl failed"; tail -5 $O/prof_$wl.err; exit 1; }
done
echo prof ok
