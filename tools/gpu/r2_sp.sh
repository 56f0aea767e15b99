cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2sp
mkdir -p $O
timeout -k 10 120 ./tools/lab/bin/scatter_probe > $O/probe.json 2>&1 && cat $O/probe.json &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $O/pmc -o run --output-format csv -- ./tools/lab/bin/scatter_probe > $O/pmc.log 2>&1
echo rc=$?
