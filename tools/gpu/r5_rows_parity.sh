#!/bin/bash
# bench.next_rows() with the rows' own parity (leader / ReadIndex at 256K
# groups vs the C oracle, wire over all 16M messages vs the C decoder, conf
# change checked whole on the device, the composed row's decode + state).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -c "import json, bench; print(json.dumps(bench.next_rows()))" \
  > $O/next_rows.json 2> $O/next_rows.err || { tail -20 $O/next_rows.err; exit 1; }
python3 -c "
import json; rows=json.load(open('$O/next_rows.json'))
for r in rows: print(r.get('config'), round(r.get('per_launch_us',0),1), r.get('parity', r.get('error')))"
