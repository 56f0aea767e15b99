#!/bin/bash
# A/B of bench.py variants on the default workload (configs[1]) with the
# driver's command line: alternating processes, ROUNDS rounds.
#   tools/gpu/ab_default.sh OUT ROUNDS "argsA" "argsB" ...   (args comma-separated)
set -o pipefail
O=${1:?out}; R=$2; shift 2; mkdir -p $O
for i in $(seq $R); do
  for v in "$@"; do
    a=${v//,/ }
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $a \
      > $O/b.json 2> $O/b.err || { echo "FAILED $a"; tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v'.ljust(28), 'us', round(r['avg_kernel_us'],3), 'wall_us', round(d['ms_per_step']*1e3,3), 'frac', round(r['frac'],4), 'G/s', round(d['value']/1e9,1), d['parity'][:20])" | tee -a $O/ab.log
  done
done
