# Per-kernel traces of the tracker step: perm+xcd (tree), perm without the
# XCD-major K5, and the previous layout; plus FETCH/WRITE passes of each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2p2
mkdir -p $O
for v in tree perm_noxcd noperm; do
  if [ $v = tree ]; then lp=""; else lp=$PWD/tools/lab/ab/$v.so; fi
  QB_LIB_PATH=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 200 > $O/tr_$v.json 2> $O/tr_$v.err || exit 1
  QB_LIB_PATH=$lp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/f_$v.log 2>&1 || exit 1
  QB_LIB_PATH=$lp timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o run -- python3 bench.py --workload tracker --no-cpu-baseline --preroll-ms 0 --steps 8 --warmup 2 > $O/w_$v.log 2>&1 || exit 1
done
echo rc=$?
