# K5 write-back granularity: tree = whole wave segments for match rows,
# committed and active (QB_K5_FULL=2); full1 = committed/active only; full0
# = changed lanes only; *nt = nontemporal stores; head = HEAD.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2wb
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker tree full1 full0 full2nt full0nt head > $O/ab.log 2>&1
echo rc=$?
