cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2fl
mkdir -p $O
F=product,ldsdma2_b512,ldsdma4_nt,ldsdma4_b512,ldsdma4_b128,ldsdma8_b128,ldsdma8_nt,ldsdma4_aux1
timeout -k 10 200 python3 -u tools/lab/run_fixed_lab.py --focus $F --rounds 9 > $O/focus_1m.log 2>&1 &&
timeout -k 10 200 python3 -u tools/lab/run_fixed_lab.py --focus $F --rounds 5 --groups 16777216 --batches 2 > $O/focus_16m.log 2>&1
echo rc=$?
