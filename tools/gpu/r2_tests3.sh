cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_votes.py tests/test_gpu_abi_raw.py tests/test_gpu_shard.py > gpurun_out/r2c_tests3.log 2>&1
echo rc=$?
