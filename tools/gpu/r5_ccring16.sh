#!/bin/bash
# Lab: k_cc_move with the inflight ring (K = 4) moved as two 16-byte loads
# (tools/lab/ab/ccring16.so) against the tree on the conf-change row, plus
# the lab build's whole-output check.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
for v in ccring16; do
timeout -k 10 300 python3 -u -c "
import sys; sys.path.insert(0, 'tools')
from etcd_amd import _lib; _lib.use_lab_library('tools/lab/ab/$v.so')
import bench_configs as b
b.confchange_config(1 << 23, 2, reporter=lambda *a: print('$v', a[-1].get('parity')), gpu_only=True)
" > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
bash tools/lab/ab_rows.sh 3 confchange tree ccring16 > $O/ab_confchange_ring16.log 2>&1 || exit 1
grep -o '^[a-z0-9]* \|per_launch_us": [0-9.]*\|"parity": "[^"]*"' $O/ab_confchange_ring16.log
