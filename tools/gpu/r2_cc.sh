cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_confchange.py > $O/tests.log 2>&1 && \
timeout -k 10 600 bash tools/lab/ab_rows.sh 2 confchange tree base > $O/ab_cc.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cc_trace -o run -- python3 tools/bench_configs.py --only confchange --reps 10 --gpu-only > $O/cc_trace.jsonl 2> $O/cc_trace.err
echo rc=$?
