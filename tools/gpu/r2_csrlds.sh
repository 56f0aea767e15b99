# CSR apply with the old run staged into the LDS accumulator (tree; + an
# SGPR cap: csr_cap) vs the register form (csr_reg): parity, A/B, trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2cl
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker_csr.py tests/test_gpu_abi_raw.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker-csr tree csr_cap csr_reg > $O/ab.log 2>&1 || exit 1
QB_LIB_PATH= timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_tree -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline > $O/tr_tree.json 2> $O/tr_tree.err
echo rc=$?
