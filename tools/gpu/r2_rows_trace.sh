# Per-kernel traces of the §8f rows (leader step, ReadIndex, wire ingest).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2rows
mkdir -p $O
for w in leader readindex wire; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$w -o run -- python3 tools/bench_configs.py --only $w --gpu-only --reps 20 > $O/tr_$w.log 2>&1 || exit 1
done
echo rc=$?
