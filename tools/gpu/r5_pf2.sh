#!/bin/bash
# Leader step: the first run and max_ents prefetched too — leader tests and
# leader / ReadIndex A/B against the committed build (pf1).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/run.sh $O tests:test_gpu_leader.py || exit 1
bash tools/lab/ab_rows.sh 3 leader tree pf1 > $O/ab_leader.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 3 readindex tree pf1 > $O/ab_readindex.log 2>&1 || exit 1
cat $O/ab_leader.log $O/ab_readindex.log
