# §8f rows: kernel trace + FETCH_SIZE / WRITE_SIZE passes per row (development).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r2rows}
mkdir -p $O
for row in ${ROWS:-leader wire confchange}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${row}_trace -o run -- python3 tools/bench_configs.py --only $row --reps 10 --gpu-only > $O/${row}_trace.jsonl 2> $O/${row}_trace.err || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${row}_fetch -o run -- python3 tools/bench_configs.py --only $row --reps 4 --gpu-only > $O/${row}_fetch.log 2>&1 || exit 2
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${row}_write -o run -- python3 tools/bench_configs.py --only $row --reps 4 --gpu-only > $O/${row}_write.log 2>&1 || exit 3
done
echo rc=0
