cd $GRAFT_REPO_ROOT
set -o pipefail
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_tracker.py > gpurun_out/r2t_tests.log 2>&1 && \
timeout -k 10 200 python3 bench.py --workload tracker > gpurun_out/r2t_bench.json 2> gpurun_out/r2t_bench.err && \
timeout -k 10 100 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2t_fixed.json 2> gpurun_out/r2t_fixed.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2t_prof -o run -- python3 bench.py --workload tracker --no-cpu-baseline > gpurun_out/r2t_prof.log 2>&1
echo rc=$?
