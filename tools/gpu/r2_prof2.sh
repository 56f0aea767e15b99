cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2q
K="k_bk_hist,k_scan_local,k_bk_sums_parts,k_bk_scatter,k_bk_split,k_csr_apply,k_bk_slow"
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_leader.py > gpurun_out/r2q/leader_tests.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2q/fixed_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2q/fixed_trace_bench.json 2> gpurun_out/r2q/fixed_trace.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2q/csr_trace -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline > gpurun_out/r2q/csr_trace_bench.json 2> gpurun_out/r2q/csr_trace.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2q/csr_fetch -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2q/csr_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2q/csr_write -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2q/csr_write.log 2>&1
echo rc=$?
