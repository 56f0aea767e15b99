#!/bin/bash
# The tracker step standalone vs inside the default run (development tool).
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload tracker --no-cpu-baseline > /tmp/t1.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('/tmp/t1.json').read().strip().splitlines()[-1]); print('standalone', round(d['roofline']['avg_kernel_us'],1), flush=True)"
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > /tmp/t2.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('/tmp/t2.json').read().strip().splitlines()[-1]); o=d['other_configs']
print('default-run', round(o['tracker']['roofline']['avg_kernel_us'],1), 'csr', round(o['tracker-csr']['roofline']['avg_kernel_us'],1), flush=True)"
done
