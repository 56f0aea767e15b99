cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r2f}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] && timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo rc=$?
