cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2f
timeout -k 10 1200 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2f/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f/smoke.log 2>&1 && \
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2f/bench_driver_cmd.json 2> gpurun_out/r2f/bench_driver_cmd.err && \
timeout -k 10 120 python3 bench.py > gpurun_out/r2f/bench_default.json 2> gpurun_out/r2f/bench_default.err && \
timeout -k 10 200 python3 bench.py --workload tracker > gpurun_out/r2f/bench_tracker.json 2> gpurun_out/r2f/bench_tracker.err && \
timeout -k 10 200 python3 bench.py --workload tracker-csr > gpurun_out/r2f/bench_tracker_csr.json 2> gpurun_out/r2f/bench_tracker_csr.err && \
timeout -k 10 200 python3 bench.py --workload ragged > gpurun_out/r2f/bench_ragged.json 2> gpurun_out/r2f/bench_ragged.err && \
timeout -k 10 200 python3 bench.py --workload joint > gpurun_out/r2f/bench_joint.json 2> gpurun_out/r2f/bench_joint.err
echo rc=$?
