cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2q2
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/csr_sq1 -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 6 --warmup 2 > $O/csr_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $O/csr_sq2 -o run -- python3 bench.py --workload tracker-csr --no-cpu-baseline --preroll-ms 0 --steps 6 --warmup 2 > $O/csr_sq2.log 2>&1
echo rc=$?
