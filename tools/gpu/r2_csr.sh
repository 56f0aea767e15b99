cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tracker_csr.py tests/test_gpu_abi_raw.py > $O/tests.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker-csr tree csrch512cap8 base > $O/ab_csr2.log 2>&1
echo rc=$?
