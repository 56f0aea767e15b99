cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wire.py > $O/tests4.log 2>&1 && \
for i in 1 2 3; do timeout -k 10 200 python3 tools/bench_configs.py --only wire,wire-rows --reps 10 --gpu-only >> $O/wire_rows.jsonl 2>&1 || exit 1; done
echo rc=$?
