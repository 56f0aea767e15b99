cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/lab/ab_tracker.sh 3 tracker tree k5vec k3direct ch1024 > gpurun_out/r2_ab1.log 2>&1
echo rc=$?
