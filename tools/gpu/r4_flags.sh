#!/bin/bash
# Round 4: the chunk-flag fix — the new garbage-workspace test against the
# previous build (tools/lab/ab/head.so: expected to fail for fill 0x03), then
# the tracker suites on the tree.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 - > $O/garbage_head.log 2>&1 <<'PY'
from etcd_amd import _lib
_lib.use_lab_library("tools/lab/ab/head.so")
import tests.test_gpu_tracker as t
for fill in (0x01, 0x03, 0xFF):
    try:
        t.test_garbage_workspace_sends_no_chunk_to_the_slow_path(fill)
        print(f"head.so fill {fill:#04x}: passed")
    except AssertionError as e:
        print(f"head.so fill {fill:#04x}: FAILED ({e})")
PY
cat $O/garbage_head.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tracker_tests.log 2>&1 || { echo "tracker tests failed"; tail -30 $O/tracker_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/tracker_tests.log)"
