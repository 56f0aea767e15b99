cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2w
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wire.py > gpurun_out/r2w/tests.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_rows.sh 3 wire tree wirectx > gpurun_out/r2w/ab_wire2.log 2>&1
echo rc=$?
