#!/bin/bash
# End-of-round evidence on the final tree, in one GPU call: box info, the GPU
# suite, smoke(), the driver's command (and its kernel trace), and the
# FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic (the headline and
# both tracker steps at the default group terms).  The first failure ends it.
#   tools/gpu/final.sh OUTDIR
set -o pipefail
O=${1:?outdir}; mkdir -p $O/pmc; export TMPDIR=/tmp
bash tools/gpu/run.sh $O info tests smoke || exit 1
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { echo "bench failed"; tail -20 $O/bench_driver_cmd.err; exit 1; }
echo "driver command ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/driver_trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/driver_cmd_under_rocprof.json 2> $O/driver_trace.err || { echo "trace failed"; exit 1; }
echo "driver trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc/headline_$c -o run -- \
    python3 bench.py --no-cpu-baseline --no-parity --no-others --preroll-ms 0 --settle-ms 0 --steps 20 --warmup 5 \
    > $O/pmc/headline_$c.log 2>&1 || { echo "pmc headline $c failed"; exit 1; }
done
echo "headline pmc ok"
bash tools/gpu/pmc_tracker.sh $O/pmc || exit 1
