set -e
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2b_drv_$i.json 2>gpurun_out/r2b_drv_$i.err; done
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --preroll-ms 0 --no-cpu-baseline > gpurun_out/r2b_drv_nopre.json 2>&1
timeout -k 10 120 python3 bench.py --steps 1000 --warmup 200 --no-cpu-baseline > gpurun_out/r2b_k1000.json 2>&1
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --streams 1 --no-cpu-baseline > gpurun_out/r2b_s1.json 2>&1
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --streams 3 --no-cpu-baseline > gpurun_out/r2b_s3.json 2>&1
