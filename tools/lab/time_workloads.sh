#!/bin/bash
# Wall time of each bench workload (development tool).
for wl in fixed ragged joint tracker tracker-csr; do
  s=$(date +%s.%N)
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline --steps 20 > /tmp/tw.json 2>/dev/null || echo "$wl failed"
  e=$(date +%s.%N)
  python3 -c "
import json; d=json.loads(open('/tmp/tw.json').read().strip().splitlines()[-1])
print('$wl', 'wall_s', round($e-$s,1), 'frac', round(d['roofline']['frac'],4), 'parity', d.get('parity','')[:40], flush=True)"
done
