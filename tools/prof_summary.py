#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV for the judged profiles/ folder.

For every kernel name: dispatch count, mean/median/min dispatch duration, and
for runs of back-to-back dispatches (gap < --gap-us between one dispatch's
start and the previous run's end) the pipelined interval = run span / count,
which is what bench.py's region timing measures when launches overlap on
several streams.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [--filter k_fixed]
"""
import argparse
import csv
import json
import sys

import numpy as np


def summarise(path, filt="", gap_us=50.0):
    rows = [r for r in csv.DictReader(open(path)) if filt in r["Kernel_Name"]]
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]),
                                                     int(r["End_Timestamp"])))
    out = {}
    for name, iv in by.items():
        iv.sort()
        st = np.array([a for a, _ in iv], dtype=np.int64)
        en = np.array([b for _, b in iv], dtype=np.int64)
        dur = (en - st) / 1e3
        runs, cur = [], [0]
        last_end = en[0]
        for i in range(1, len(iv)):
            if (st[i] - last_end) / 1e3 > gap_us:
                runs.append(cur)
                cur = []
            cur.append(i)
            last_end = max(last_end, en[i])
        runs.append(cur)
        run_info = []
        for rr in runs:
            span = (en[rr].max() - st[rr].min()) / 1e3
            run_info.append({"dispatches": len(rr), "span_us": round(span, 2),
                             "interval_us": round(span / len(rr), 3),
                             "mean_dispatch_us": round(float(dur[rr].mean()), 3)})
        out[name] = {
            "dispatches": len(iv),
            "mean_us": round(float(dur.mean()), 3),
            "median_us": round(float(np.median(dur)), 3),
            "min_us": round(float(dur.min()), 3),
            "runs": run_info,
        }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--filter", default="")
    ap.add_argument("--gap-us", type=float, default=50.0)
    a = ap.parse_args()
    json.dump(summarise(a.trace, a.filter, a.gap_us), sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
