cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2p
mkdir -p $O
QB_LIB_PATH=$PWD/tools/lab/ab/k5p.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_abi_raw.py tests/test_gpu_shard.py > $O/tests_k5p.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker tree k5p > $O/ab_k5p.log 2>&1
echo rc=$?
