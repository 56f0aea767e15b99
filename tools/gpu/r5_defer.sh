#!/bin/bash
# Lab: the ReadIndex responses stored after the group's last record instead
# of where advance releases them (tools/lab/ab/defer.so) against the tree —
# the row parity of the lab build against the C oracle, then A/B on the
# ReadIndex and leader rows.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "
import sys; sys.path.insert(0, 'tools')
from etcd_amd import _lib; _lib.use_lab_library('tools/lab/ab/defer.so')
import bench_configs as b
print('readindex', b.leader_row_parity('readindex')); print('leader', b.leader_row_parity('leader'))
" > $O/parity_defer.log 2>&1 || { tail -20 $O/parity_defer.log; exit 1; }
cat $O/parity_defer.log
bash tools/lab/ab_rows.sh 3 readindex tree defer > $O/ab_readindex_defer.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 leader tree defer > $O/ab_leader_defer.log 2>&1 || exit 1
grep -o '^[a-z]* \|per_launch_us": [0-9.]*' $O/ab_*.log
