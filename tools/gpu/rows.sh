#!/bin/bash
# SURVEY §8f rows (tools/bench_configs.py): kernel trace + FETCH_SIZE and
# WRITE_SIZE passes per row; summarise with tools/rows_pmc.py <out> <row>.
#   tools/gpu/rows.sh OUT "leader readindex wire confchange"
set -o pipefail
O=${1:?out}; ROWS=${2:-leader readindex wire confchange}
mkdir -p $O; export TMPDIR=/tmp
for row in $ROWS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${row}_trace -o run -- \
    python3 tools/bench_configs.py --only $row --reps 10 --gpu-only > $O/${row}_trace.jsonl 2> $O/${row}_trace.err || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${row}_fetch -o run -- \
    python3 tools/bench_configs.py --only $row --reps 4 --gpu-only > $O/${row}_fetch.log 2>&1 || exit 2
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${row}_write -o run -- \
    python3 tools/bench_configs.py --only $row --reps 4 --gpu-only > $O/${row}_write.log 2>&1 || exit 3
  echo "$row ok"
done
