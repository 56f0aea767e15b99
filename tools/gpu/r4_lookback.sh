#!/bin/bash
# Round 4: k_ld_chunk_runs takes each chunk's base by a ticket-ordered
# decoupled look-back (no totals kernel, no three-kernel scan) — the leader
# GPU tests, then alternating-process A/B against HEAD (tools/lab/ab/head.so).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_leader.py tests/test_gpu_wire.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/leader_tests.log 2>&1 || { echo "leader tests failed"; tail -30 $O/leader_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/leader_tests.log)"
for row in leader readindex; do
  timeout -k 10 600 bash tools/lab/ab_rows.sh 3 $row head tree > $O/ab_$row.log 2>&1 || { echo "ab $row failed"; cat $O/ab_$row.log; exit 1; }
done
python3 - $O <<'PY'
import json, sys
for f in ("ab_leader.log", "ab_readindex.log"):
    for line in open(f"{sys.argv[1]}/{f}"):
        name, _, js = line.partition(" ")
        try:
            d = json.loads(js)
            print(f, name, round(d["per_launch_us"], 1), round(d.get("ordered_us", 0), 1))
        except Exception:
            print(f, line.strip())
PY
