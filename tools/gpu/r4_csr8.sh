#!/bin/bash
# Round 4: the CSR apply at 8 waves per SIMD (u32-saturated group terms in
# LDS: 39.5 KB, SGPRs capped at 80) — the CSR tracker tests, then
# alternating-process A/B of the CSR tick against HEAD (head.so).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tracker_csr.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
echo "tests ok: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 600 bash tools/lab/ab_tracker.sh 3 tracker-csr head tree > $O/ab_tracker_csr.log 2>&1 || { cat $O/ab_tracker_csr.log; exit 1; }
cat $O/ab_tracker_csr.log
