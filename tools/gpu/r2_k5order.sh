cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2k
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py tests/test_gpu_abi_raw.py > gpurun_out/r2k/tests2.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker tree activeonly base > gpurun_out/r2k/ab_tracker2.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker-csr tree activeonly base > gpurun_out/r2k/ab_tracker_csr2.log 2>&1
echo rc=$?
