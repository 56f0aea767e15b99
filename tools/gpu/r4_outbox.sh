#!/bin/bash
# Round 4: the leader step's per-group outbox (qb_dev_leader_step_outbox) —
# leader GPU tests, the capacity tests, then the §8f leader / ReadIndex rows
# (both forms timed in one process) and an A/B against the round-3 build.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_leader.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/leader_tests.log 2>&1 || { echo "leader tests failed"; tail -30 $O/leader_tests.log; exit 1; }
echo "leader tests ok: $(tail -1 $O/leader_tests.log)"
timeout -k 10 300 python -u tools/bench_configs.py --only leader,readindex --gpu-only > $O/rows.jsonl 2> $O/rows.err \
  || { echo "rows failed"; tail -20 $O/rows.err; exit 1; }
cat $O/rows.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_capacity.py -m gpu -x -v --timeout 600 --timeout-method thread \
  > $O/capacity_tests.log 2>&1 || { echo "capacity tests failed"; tail -40 $O/capacity_tests.log; exit 1; }
echo "capacity ok: $(tail -1 $O/capacity_tests.log)"
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    --deselect tests/test_gpu_capacity.py > $O/gpu_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_suite.log; exit 1; }
  echo "suite ok: $(tail -1 $O/gpu_suite.log)"
fi
