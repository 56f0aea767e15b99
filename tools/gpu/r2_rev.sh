# K5 chunks in reverse order (tree: consume K4's most recent output first,
# MALL reuse) vs forward (fwd): parity, A/B, FETCH pass.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2rv
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tracker.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker tree fwd > $O/ab.log 2>&1 || exit 1
QB_LIB_PATH= timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_tree -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/f_tree.log 2>&1
echo rc=$?
