# Conf change write pass and copy in reverse order (tree) vs forward (ccfwd).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2ccr
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_confchange.py tests/test_gpu_leader.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_libs.sh confchange 3 tree ccfwd > $O/ab.log 2>&1
echo rc=$?
