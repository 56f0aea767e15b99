cd $GRAFT_REPO_ROOT
timeout -k 10 100 python3 tools/lab/sync_overhead.py && \
QB_LAB_DEVFLAGS=1 timeout -k 10 100 python3 tools/lab/sync_overhead.py && \
QB_LAB_DEVFLAGS=2 timeout -k 10 100 python3 tools/lab/sync_overhead.py
