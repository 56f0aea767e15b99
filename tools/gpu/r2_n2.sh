cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r2n}
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > $O/n2_fixed.json 2> $O/n2_fixed.err
echo "fixed rc=$?"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload tracker --steps 10 --warmup 3 --backend gloo > $O/n2_tracker.json 2> $O/n2_tracker.err
echo "tracker rc=$?"
