# Launch streams at the driver's command (K = 20, W = 5): 2 (default) vs 3 vs 4,
# interleaved, three rounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2st
mkdir -p $O
for i in 1 2 3; do
  for S in 2 3 4; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams $S --no-cpu-baseline > $O/s${S}_$i.json 2> $O/s${S}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/s${S}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams=$S', round(r['avg_kernel_us'],2), round(d['ms_per_step']*1e3,2), round(r['frac'],4), flush=True)" >> $O/ab.log
  done
done
echo rc=$?
