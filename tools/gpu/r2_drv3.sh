# The driver's bench command three times on one box (variance check after an
# anomalous 0.41 line), then the default line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2d3
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || exit 1
done
timeout -k 10 200 python3 bench.py > $O/default.json 2> $O/default.err
echo rc=$?
