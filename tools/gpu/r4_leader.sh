#!/bin/bash
# Round 4: leader step with the message placement fused into k_ld_step —
# the GPU suite's leader tests, then alternating-process A/B against the
# round-3 build (tools/lab/ab/base.so) on the leader and ReadIndex rows.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_leader.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/leader_tests.log 2>&1 || { echo "leader tests failed"; tail -30 $O/leader_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/leader_tests.log)"
timeout -k 10 600 bash tools/lab/ab_rows.sh 3 leader base tree > $O/ab_leader.log 2>&1 || { echo "ab leader failed"; cat $O/ab_leader.log; exit 1; }
timeout -k 10 600 bash tools/lab/ab_rows.sh 3 readindex base tree > $O/ab_readindex.log 2>&1 || { echo "ab readindex failed"; cat $O/ab_readindex.log; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("ab_leader.log", "ab_readindex.log"):
    for line in open(f"{sys.argv[1]}/{f}"):
        name, _, js = line.partition(" ")
        try:
            d = json.loads(js)
            print(f, name, round(d["per_launch_us"], 1), round(d["frac_hbm_peak"], 3))
        except Exception:
            print(f, line.strip())
PY
