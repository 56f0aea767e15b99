#!/bin/bash
# Round 4: the configs[1] line at 2, 3 and 4 launch streams, alternated (one
# process per run; only the headline workload, --workload default).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for s in 2 3 4 1; do
    timeout -k 10 300 python -u bench.py --streams $s --no-others --no-cpu-baseline > $O/s${s}_r${rep}.json 2> $O/s${s}_r${rep}.err \
      || { echo "streams $s failed"; tail -20 $O/s${s}_r${rep}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['achieved'], r['frac'], d.get('value_mall_warm'))" $O/s${s}_r${rep}.json "streams=$s rep=$rep"
  done
done
