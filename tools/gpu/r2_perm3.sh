# Interleaved super-buckets (perm mode, linear K5): parity, then per-kernel
# traces and traffic of tree / perm_xcd / noperm.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2p3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py tests/test_gpu_tracker_csr.py > $O/tests.log 2>&1 || exit 1
for v in tree perm_xcd noperm; do
  if [ $v = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$v.so; fi
  QB_LIB_PATH=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 200 > $O/tr_$v.json 2> $O/tr_$v.err || exit 1
done
QB_LIB_PATH= timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/f_tree.log 2>&1 || exit 1
QB_LIB_PATH= timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/w_tree.log 2>&1 || exit 1
timeout -k 10 600 bash tools/lab/ab_tracker.sh 2 tracker-csr tree noperm > $O/ab_csr.log 2>&1
echo rc=$?
