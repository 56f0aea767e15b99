# LDS-DMA fixed kernel: parity, driver-command bench lines, trace, PMC traffic.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2fx
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_quorum.py tests/test_gpu_abi_raw.py tests/test_gpu_shard.py > $O/tests.log 2>&1 && \
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv1.json 2> $O/e1.err && \
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv2.json 2> $O/e2.err && \
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv3.json 2> $O/e3.err && \
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/default.json 2> $O/e4.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --no-cpu-baseline --preroll-ms 0 --steps 50 --warmup 5 > $O/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --no-cpu-baseline --preroll-ms 0 --steps 50 --warmup 5 > $O/write.log 2>&1
echo rc=$?
