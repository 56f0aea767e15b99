# Leader step slot-stage write-back as whole wave segments (tree) vs HEAD
# (dirty slots only): parity, then interleaved A/B of the leader and
# ReadIndex workloads.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2ld
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_leader.py tests/test_gpu_tracker_csr.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_libs.sh leader,readindex 3 tree head > $O/ab.log 2>&1
echo rc=$?
