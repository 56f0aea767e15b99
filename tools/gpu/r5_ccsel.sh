#!/bin/bash
# k_cc_move with one load / store per column for carried and fresh lanes (the
# tree) against the 16-byte-ring build before it (tools/lab/ab/ring16.so):
# the conf-change GPU suite, the row's whole-output check, then A/B.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_confchange.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests_confchange.log 2>&1 || { tail -30 $O/gpu_tests_confchange.log; exit 1; }
tail -1 $O/gpu_tests_confchange.log
timeout -k 10 300 python3 -u -c "
import sys; sys.path.insert(0, 'tools')
import bench_configs as b
b.confchange_config(1 << 23, 2, reporter=lambda *a: print('tree', a[-1].get('parity')), gpu_only=True)
" > $O/parity_tree.log 2>&1 || { tail -20 $O/parity_tree.log; exit 1; }
tail -1 $O/parity_tree.log
bash tools/lab/ab_rows.sh 3 confchange tree ring16 > $O/ab_confchange_select.log 2>&1 || exit 1
grep -o '^[a-z0-9]* \|per_launch_us": [0-9.]*' $O/ab_confchange_select.log
