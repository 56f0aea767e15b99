# Wire ingest: the deferred launch's status scan as one 16-byte load per
# thread (tree) vs HEAD: parity, A/B, trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2wd
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wire.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_libs.sh wire 3 tree head > $O/ab.log 2>&1 || exit 1
QB_LIB_PATH= timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_tree -o run -- python3 tools/bench_configs.py --only wire --gpu-only --reps 20 > $O/tr_tree.log 2>&1
echo rc=$?
