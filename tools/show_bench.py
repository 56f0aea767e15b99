#!/usr/bin/env python3
"""Print the key fields of bench.py JSON lines found in the given log files."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = [l for l in open(path) if l.startswith("{")]
    except OSError as e:
        print(path, "missing", e)
        continue
    for l in lines:
        d = json.loads(l)
        r = d["roofline"]
        cb = d.get("cpu_baseline") or {}
        print(f"{path}: value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.4f}  "
              f"kern {r['avg_kernel_us']:.2f}us  {r['achieved']:.0f} GB/s frac {r['frac']:.3f}  "
              f"warm {d.get('value_mall_warm', 0):.4g}  cpu {cb.get('value', 0):.4g}  "
              f"ag {d.get('allgather_ms')}")
