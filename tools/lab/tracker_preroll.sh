#!/bin/bash
# The standalone tracker step after pre-rolls of different length (development tool).
for i in 1 2; do for p in 300 3000 8000; do
  timeout -k 10 300 python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms $p > /tmp/t1.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('/tmp/t1.json').read().strip().splitlines()[-1]); print('preroll $p', round(d['roofline']['avg_kernel_us'],1), d['preroll_steps'], flush=True)"
done; done
