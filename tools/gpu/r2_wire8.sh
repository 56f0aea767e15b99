cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2w8
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_leader.py > $O/tests.log 2>&1 && \
timeout -k 10 400 bash tools/lab/ab_rows.sh 3 wire tree base > $O/ab.log 2>&1 && \
timeout -k 10 400 bash tools/lab/ab_rows.sh 2 wire-csr tree base > $O/ab_csr.log 2>&1
echo rc=$?
