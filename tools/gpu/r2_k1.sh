cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2k1
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py tests/test_gpu_leader.py > $O/tests.log 2>&1 && \
QB_LIB_PATH=$PWD/tools/lab/ab/k1t4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tracker.py > $O/tests_t4.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker tree k1t4 base > $O/ab_k1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_trace -o run -- python3 bench.py --workload tracker --no-cpu-baseline > $O/tr_trace.json 2> $O/tr_trace.err
echo rc=$?
