#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE in separate runs of the same command): median per dispatch,
FETCH_SIZE doubled (gfx950 wide-read correction, MI355X_MICROARCH.md),
KiB -> MB.  Development tool.

    python tools/pmc_kernels.py D1/run_counter_collection.csv D2/run_counter_collection.csv [filter]
"""
import collections
import csv
import sys

import numpy as np


def load(path, counter):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = r["Kernel_Name"]
        d = int(r["Dispatch_Id"])
        per[k][d] = per[k].get(d, 0.0) + float(r["Counter_Value"])
    return {k: float(np.median(list(v.values()))) for k, v in per.items()}


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    flt = sys.argv[3] if len(sys.argv) > 3 else ""
    print(f"{'kernel':60s} {'read MB':>9s} {'write MB':>9s}")
    for k in sorted(set(f) | set(w)):
        if flt not in k:
            continue
        rd = 2 * f.get(k, 0.0) * 1024 / 1e6
        wr = w.get(k, 0.0) * 1024 / 1e6
        print(f"{k[:60]:60s} {rd:9.1f} {wr:9.1f}")


if __name__ == "__main__":
    main()
