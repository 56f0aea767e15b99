# Interleaved super-buckets without the permutation (tree) vs the previous
# layout (noperm) and perm+il: parity, traces, interleaved A/B on both steps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2il
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py > $O/tests.log 2>&1 || exit 1
QB_LIB_PATH= timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 200 > $O/tr_tree.json 2> $O/tr_tree.err || exit 1
QB_LIB_PATH= timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/f_tree.log 2>&1 || exit 1
QB_LIB_PATH= timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/w_tree.log 2>&1 || exit 1
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker tree noperm perm_il > $O/ab.log 2>&1 || exit 1
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker-csr tree noperm > $O/ab_csr.log 2>&1
echo rc=$?
