cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2l
mkdir -p $O
QB_LIB_PATH=$PWD/tools/lab/ab/ldw5.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_leader.py > $O/tests_ldw5.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_rows.sh 2 leader tree ldspan1280 ldw5 > $O/ab_ld2.log 2>&1 && \
timeout -k 10 400 bash tools/lab/ab_rows.sh 2 readindex tree ldw5 > $O/ab_ri2.log 2>&1
echo rc=$?
