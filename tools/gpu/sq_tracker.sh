#!/bin/bash
# SQ / TCC counters of the tracker kernels (one pass per counter group).
set -o pipefail
O=${1:?out}; WL=${2:-tracker}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- \
    python3 bench.py --workload $WL --no-cpu-baseline --no-parity --preroll-ms 0 --steps 6 --warmup 2 \
    > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }
  echo "$n ok"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum
