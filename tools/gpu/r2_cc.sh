# Conf change: fresh Progress rows materialised by k_cc_copy (every new
# slot's row written there, whole lines) vs the write pass storing them
# (cc_base): parity, A/B, per-kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2cc
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_confchange.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/lab/ab_libs.sh confchange 3 tree cc_base > $O/ab.log 2>&1 || exit 1
QB_LIB_PATH= timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_tree -o run -- python3 tools/bench_configs.py --only confchange --gpu-only --reps 20 > $O/tr_tree.log 2>&1
echo rc=$?
