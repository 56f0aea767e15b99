for i in 1 2 3; do for s in 2 3 4; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams $s --no-cpu-baseline > /tmp/s.json 2>/dev/null && python3 -c "
import json; d=json.loads(open('/tmp/s.json').read().strip().splitlines()[-1]); r=d['roofline']
print('streams $s', 'value', round(d['value']/1e9,1), 'wall_us', round(d['ms_per_step']*1e3,2), 'kern_us', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],4), flush=True)"
done; done
