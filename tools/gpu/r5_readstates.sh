#!/bin/bash
# The outbox's ReadState area: the leader GPU suite (incl. the new
# read-state fuzz and the 256K ReadIndex workload vs the C oracle), then the
# ReadIndex row with all three forms timed in one process and its own parity.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_leader.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests_leader.log 2>&1 || { tail -30 $O/gpu_tests_leader.log; exit 1; }
tail -2 $O/gpu_tests_leader.log
timeout -k 10 300 python3 -u -c "
import sys, json; sys.path.insert(0, 'tools')
import bench_configs as b
b.readindex_config(1 << 22, 10, reporter=lambda name, G, t, algo, extra: print(json.dumps(
    dict(config=name, per_launch_us=t * 1e6, algo=algo, frac=algo / t / 1e9 / b.HBM_PEAK_GBS, **extra))),
    gpu_only=True)
" > $O/readindex_row.json 2> $O/readindex_row.err || { tail -20 $O/readindex_row.err; exit 1; }
cat $O/readindex_row.json
