# CSR apply chunks in reverse order (tree) vs forward (csrfwd).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2crv
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker_csr.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker-csr tree csrfwd > $O/ab.log 2>&1
echo rc=$?
