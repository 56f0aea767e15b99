# Pipelined ticks (bucket k+1 on a side stream while k is applied) vs one
# step call per tick: parity test, then interleaved bench runs and a trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2pp
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for p in 1 0; do
    timeout -k 10 200 python3 bench.py --workload tracker --no-cpu-baseline --pipeline $p > $O/b_${p}_$i.json 2> $O/b_${p}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/b_${p}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pipeline=$p', round(r['avg_kernel_us'],1), round(d['ms_per_step']*1e3,1), round(r['frac'],4), flush=True)" >> $O/ab.log
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_pipe -o run -- python3 bench.py --workload tracker --no-cpu-baseline > $O/tr_pipe.json 2> $O/tr_pipe.err
echo rc=$?
