# Perm-mode level 2 (K4 writes a permutation, K5 gathers): tracker parity,
# then interleaved A/B against the previous layout (noperm.so).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_abi_raw.py > $O/tests.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker tree noperm > $O/ab.log 2>&1
echo rc=$?
