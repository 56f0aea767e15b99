#!/bin/bash
# Round 4: the conf change's scan add-back folded into the write pass — the
# conf change tests, then alternating-process A/B against HEAD (head.so).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_confchange.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 600 bash tools/lab/ab_rows.sh 3 confchange head tree > $O/ab_confchange.log 2>&1 || { cat $O/ab_confchange.log; exit 1; }
python3 - $O <<'PY'
import json, sys
for line in open(f"{sys.argv[1]}/ab_confchange.log"):
    name, _, js = line.partition(" ")
    try:
        print(name, round(json.loads(js)["per_launch_us"], 1))
    except Exception:
        print(line.strip())
PY
