# CSR apply at 4 workgroups per CU (act masks packed to fit LDS, 64-VGPR
# budget) vs without the waves bound vs HEAD; fixed step re-checked.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2co
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker_csr.py > $O/tests.log 2>&1 || exit 1
QB_LIB_PATH= timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_tree -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 200 > $O/tr_tree.json 2> $O/tr_tree.err || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker-csr tree csr_nolb head > $O/ab_csr.log 2>&1
echo rc=$?
