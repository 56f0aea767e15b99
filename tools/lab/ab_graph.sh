set -e
for r in 1 2; do
for g in 0 16 64 256; do
timeout -k 10 120 python bench.py --no-cpu-baseline --graph $g > gpurun_out/g_${g}_$r.json
python -c "import json;d=json.load(open('gpurun_out/g_${g}_$r.json'));print('graph',$g,'run',$r,round(d['value']/1e9,1),'G/s kernel_us',round(d['roofline']['avg_kernel_us'],2),'frac',round(d['roofline']['frac'],3))"
done; done
timeout -k 10 300 python tools/bench_configs.py --only 1 > gpurun_out/plumbing.jsonl
