#!/bin/bash
# One parameterised GPU-box script (replaces round 2's per-experiment
# tools/gpu/r2_*.sh).  Usage: tools/gpu/run.sh OUTDIR STEP [STEP ...]
# Steps (each under its own time limit; the first failure ends the script):
#   tests            pytest -m gpu (one process)
#   tests:FILE[::K]  one GPU test file / test
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     bench.py with ARGS (commas for spaces), JSON to OUTDIR/bench_<n>.json
#                    (limit $BENCH_TIMEOUT seconds, default 400)
#   prof[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc:CTR[:ARGS]   one rocprofv3 --pmc pass (one counter group) of bench.py ARGS
#   info             host / GPU description
set -o pipefail
O=${1:?outdir}; shift
mkdir -p "$O"
export TMPDIR=/tmp
n=0
for s in "$@"; do
  n=$((n+1))
  kind=${s%%:*}; arg=${s#*:}; [ "$arg" = "$s" ] && arg=""
  args=${arg//,/ }
  case $kind in
    tests)
      if [ -n "$arg" ]; then tgt=tests/$arg; else tgt=tests; fi
      timeout -k 10 900 python -u -m pytest $tgt -m gpu -x -v --timeout 600 --timeout-method thread \
        > "$O/tests_$n.log" 2>&1 || { echo "tests failed ($?)"; tail -30 "$O/tests_$n.log"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; cat "$O/smoke.log"; exit 1; } ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $args > "$O/bench_$n.json" 2> "$O/bench_$n.err" \
        || { echo "bench $args failed"; tail -20 "$O/bench_$n.err"; exit 1; } ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$n" -o run \
        -- python3 bench.py $args > "$O/prof_$n.json" 2> "$O/prof_$n.err" \
        || { echo "prof failed"; tail -20 "$O/prof_$n.err"; exit 1; } ;;
    pmc)
      ctr=${arg%%:*}; rest=${arg#*:}; [ "$rest" = "$arg" ] && rest=""
      timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_${ctr}_$n" -o run \
        -- python3 bench.py ${rest//,/ } > "$O/pmc_${ctr}_$n.log" 2>&1 \
        || { echo "pmc $ctr failed"; tail -20 "$O/pmc_${ctr}_$n.log"; exit 1; } ;;
    info)
      { nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
        grep -m1 "model name" /proc/cpuinfo; rocm-smi --showproductname 2>/dev/null | head -20; } > "$O/info.txt" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $n ($s) ok"
done
