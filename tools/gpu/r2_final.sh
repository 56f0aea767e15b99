# End-of-session check of the committed tree: the GPU suite, smoke, and every
# bench line (driver command, default, tracker, tracker-csr, ragged, joint).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2fin
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/e1.err && \
timeout -k 10 200 python3 bench.py > $O/bench_default.json 2> $O/e2.err && \
timeout -k 10 300 python3 bench.py --workload tracker > $O/bench_tracker.json 2> $O/e3.err && \
timeout -k 10 300 python3 bench.py --workload tracker-csr > $O/bench_tracker_csr.json 2> $O/e4.err && \
timeout -k 10 200 python3 bench.py --workload ragged > $O/bench_ragged.json 2> $O/e5.err && \
timeout -k 10 200 python3 bench.py --workload joint > $O/bench_joint.json 2> $O/e6.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_trace.json 2> $O/drv_trace.err
echo rc=$?
