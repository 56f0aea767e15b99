cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2l
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_leader.py > $O/tests.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_rows.sh 3 leader tree base > $O/ab_ld.log 2>&1 && \
timeout -k 10 300 bash tools/lab/ab_rows.sh 2 readindex tree base > $O/ab_ri.log 2>&1
echo rc=$?
