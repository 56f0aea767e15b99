cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="k_bk_hist,k_scan_local,k_bk_sums_parts,k_bk_scatter,k_bk_split,k_bk_apply,k_bk_slow"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_trace -o run -- python3 bench.py --workload tracker --no-cpu-baseline > gpurun_out/r2p_trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2p_fetch -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2p_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2p_write -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2p_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/r2p_sq -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2p_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r2p_tcc -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > gpurun_out/r2p_tcc.log 2>&1 && \
python3 tools/pmc_traffic.py --fetch gpurun_out/r2p_fetch/run_counter_collection.csv --write gpurun_out/r2p_write/run_counter_collection.csv --kernel $K --warmup 2 --steps 1000 --key tracker_n5_G16777216 --algo-bytes 1694498816 --out profiles/pmc_traffic.json > gpurun_out/r2p_traffic.log 2>&1 && \
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_quorum.py -k "joint_8m or bench_test_go" > gpurun_out/r2p_qtests.log 2>&1 && \
timeout -k 10 200 python3 bench.py --workload tracker-csr > gpurun_out/r2p_csr_bench.json 2> gpurun_out/r2p_csr_bench.err
echo rc=$?
