#!/bin/bash
# A/B of library builds on the streaming tracker step (bench.py --workload
# tracker): tools/lab/ab/<name>.so per name, "tree" = the in-tree build,
# alternating processes on one box for `rounds` rounds.  Development tool.
#   ab_tracker.sh <rounds> <workload> name1 name2 ...   (env AB_ARGS: extra bench.py args)
cd "$(dirname "$0")/../.."
rounds=$1; wl=$2; shift 2
for i in $(seq $rounds); do
  for name in "$@"; do
    if [ "$name" = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$name.so; fi
    if timeout -k 10 150 python3 bench.py ${lp:+--lab-lib $lp} --workload $wl --no-cpu-baseline --preroll-ms 200 $AB_ARGS \
        > /tmp/ab_$name.json 2> /tmp/ab_$name.err; then
      python3 -c "import sys,json
d=json.loads(open('/tmp/ab_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', 'step_us', round(r['avg_kernel_us'],1), 'wall_us', round(d['ms_per_step']*1e3,1), 'frac', round(r['frac'],4), str(d.get('parity',''))[:24], flush=True)"
    else
      echo "$name FAILED rc=$?"; tail -5 /tmp/ab_$name.err
    fi
  done
done
