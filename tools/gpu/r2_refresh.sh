# Round-2 refresh after the K5 changes: bench lines, tracker traces and PMC
# traffic passes (FETCH_SIZE / WRITE_SIZE separately), then the registry.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2r
mkdir -p $O
K5="k_bk_hist,k_scan_local,k_bk_sums_parts,k_bk_scatter,k_bk_split,k_bk_apply,k_bk_slow"
KC="k_bk_hist,k_scan_local,k_bk_sums_parts,k_bk_scatter,k_bk_split,k_csr_apply<,k_csr_apply_deferred,k_bk_slow"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/e1.err && \
timeout -k 10 300 python3 bench.py --workload tracker > $O/bench_tracker.json 2> $O/e3.err && \
timeout -k 10 300 python3 bench.py --workload tracker-csr > $O/bench_tracker_csr.json 2> $O/e4.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_trace -o run -- python3 bench.py --workload tracker --no-cpu-baseline > $O/tr_trace.json 2> $O/tr_trace.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/csr_trace -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline > $O/csr_trace.json 2> $O/csr_trace.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_fetch -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/tr_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_write -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/tr_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/csr_fetch -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/csr_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/csr_write -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/csr_write.log 2>&1 && \
python3 tools/pmc_traffic.py --fetch $O/tr_fetch/run_counter_collection.csv --write $O/tr_write/run_counter_collection.csv --kernel $K5 --warmup 2 --steps 1000 --key tracker_n5_G16777216 --algo-bytes 1694498816 --out $O/pmc_traffic_tracker.json > $O/traffic_tr.log 2>&1 && \
python3 tools/pmc_traffic.py --fetch $O/csr_fetch/run_counter_collection.csv --write $O/csr_write/run_counter_collection.csv --kernel $KC --warmup 2 --steps 1000 --key tracker_csr_n5_G16777216 --algo-bytes 1962890720 --out $O/pmc_traffic_csr.json > $O/traffic_csr.log 2>&1
echo rc=$?
