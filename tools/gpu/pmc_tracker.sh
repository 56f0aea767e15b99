#!/bin/bash
# PMC traffic of the tracker steps (separate FETCH_SIZE / WRITE_SIZE passes,
# MI355X_MICROARCH.md HBM section) + a kernel trace of the CSR step.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for wl in tracker tracker-csr; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${wl}_$c -o run -- \
      python3 bench.py --workload $wl --no-cpu-baseline --no-parity --preroll-ms 0 --steps 8 --warmup 2 \
      > $O/${wl}_$c.log 2>&1 || { echo "pmc $wl $c failed"; tail -5 $O/${wl}_$c.log; exit 1; }
    echo "$wl $c ok"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_csr -o run -- \
  python3 bench.py --workload tracker-csr --no-cpu-baseline --no-parity > $O/prof_csr.json 2> $O/prof_csr.err || exit 1
echo prof ok
