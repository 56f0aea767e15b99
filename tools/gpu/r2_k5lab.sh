# Where K5's time goes: lab builds without its stores, without its record
# pass, and with neither (state loads only), per-kernel traces.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2k5
mkdir -p $O
for v in tree lab_nostore lab_norecs lab_loadsonly; do
  if [ $v = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$v.so; fi
  QB_LIB_PATH=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 200 > $O/tr_$v.json 2> $O/tr_$v.err || exit 1
done
echo rc=$?
