set -o pipefail
O=gpurun_out/r3ld; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_leader.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo tests ok
bash tools/lab/ab_rows.sh 3 readindex ldfd tree > $O/ab_ri.log 2>&1 || exit 1
cat $O/ab_ri.log
bash tools/lab/ab_rows.sh 3 leader ldfd tree > $O/ab_ld.log 2>&1 || exit 1
cat $O/ab_ld.log
bash tools/gpu/rows.sh $O "readindex leader" || exit 1
