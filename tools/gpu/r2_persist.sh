# Persistent K5 (grid = P workgroups per CU striding over the chunks): tree
# (P = 4) vs P = 3, 2, 0 (one per chunk) vs head.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2ps
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker tree p3 p2 p0 > $O/ab.log 2>&1
echo rc=$?
