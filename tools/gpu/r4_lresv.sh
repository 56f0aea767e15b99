#!/bin/bash
# Round 4: the leader's bucketing on reserved regions too (no histogram, scan
# or part table; a skewed batch's excess through the overflow area) and the
# region capacity from the tiles per XCD slot — the GPU suite, then
# alternating-process A/B against HEAD (tools/lab/ab/head.so).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/gpu_tests.log)"
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
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker head tree > $O/ab_tracker.log 2>&1 || { cat $O/ab_tracker.log; exit 1; }
cat $O/ab_tracker.log
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker-csr head tree > $O/ab_tracker_csr.log 2>&1 || { cat $O/ab_tracker_csr.log; exit 1; }
cat $O/ab_tracker_csr.log
