cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2w5
mkdir -p $O
timeout -k 10 400 bash tools/lab/ab_rows.sh 2 wire tree wirenoparse > $O/ab_noparse_rows.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/sq -o run -- python3 tools/bench_configs.py --only wire --reps 3 --gpu-only > $O/sq.log 2>&1
echo rc=$?
