cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracker_csr.py tests/test_gpu_tracker.py > gpurun_out/r2c_tests.log 2>&1
echo rc=$?
