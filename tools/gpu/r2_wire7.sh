cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2w7
mkdir -p $O
timeout -k 10 400 bash tools/lab/ab_rows.sh 2 wire tree wirenogeneric wirenoparse > $O/ab.log 2>&1
echo rc=$?
