"""Per-kernel median duration, HBM read (FETCH_SIZE x2, gfx950) and write
bytes per dispatch for one profiled run directory set (development tool).
  rows_pmc.py <dir> <row>  ->  <dir>/<row>_{trace,fetch,write}/run_*.csv"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "")[-60:]


def main():
    d, row = sys.argv[1], sys.argv[2]
    dur = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/{row}_trace/run_kernel_trace.csv")):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rd, wr = defaultdict(list), defaultdict(list)
    for kind, acc in (("fetch", rd), ("write", wr)):
        per = defaultdict(float)
        for r in csv.DictReader(open(f"{d}/{row}_{kind}/run_counter_collection.csv")):
            key = (r["Dispatch_Id"], short(r["Kernel_Name"]))
            per[key] += float(r["Counter_Value"])
        for (_, k), v in per.items():
            acc[k].append(v * 1024 * (2 if kind == "fetch" else 1))
    print(f"{'kernel':60s} {'n':>5s} {'med us':>9s} {'read MB':>9s} {'write MB':>9s} {'TB/s':>7s}")
    tot = [0.0, 0.0, 0.0]
    for k, v in sorted(dur.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
        if not k.startswith("qb::"):
            continue
        m = statistics.median(v) / 1e3
        r = statistics.median(rd[k]) / 1e6 if rd[k] else float("nan")
        w = statistics.median(wr[k]) / 1e6 if wr[k] else float("nan")
        print(f"{k:60s} {len(v):5d} {m:9.1f} {r:9.1f} {w:9.1f} {(r + w) / m:7.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
