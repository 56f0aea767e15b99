#!/bin/bash
# Round 5: escape column (K3 writes escaped records' exact index/term beside
# them) + conf change move kernel v2: GPU tests of both, A/B of the uniform
# tracker ticks and conf change vs the round-4 build, the composed wire ->
# tracker row (terms >= 1023: every record escapes); the leader step with
# first index / log bounds prefetched (leader tests, leader / ReadIndex A/B).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_confchange.py tests:test_gpu_tracker.py tests:test_gpu_tracker_csr.py tests:test_gpu_wire.py tests:test_gpu_leader.py || exit 1
bash tools/lab/ab_rows.sh 2 confchange tree base > $O/ab_confchange.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cc_prof -o run -- \
  python3 tools/bench_configs.py --only confchange --reps 10 --gpu-only > $O/cc_prof.log 2>&1 || exit 1
AB_ARGS=--no-parity bash tools/lab/ab_tracker.sh 2 tracker tree base > $O/ab_tracker.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only wire-tracker --reps 10 --gpu-only \
  > $O/wire_tracker.json 2> $O/wire_tracker.err || { tail -5 $O/wire_tracker.err; exit 1; }
bash tools/lab/ab_rows.sh 2 leader tree base > $O/ab_leader.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 readindex tree base > $O/ab_readindex.log 2>&1 || exit 1
cat $O/ab_confchange.log $O/ab_tracker.log $O/ab_leader.log $O/ab_readindex.log $O/wire_tracker.json
