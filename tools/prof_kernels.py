"""Summarise a rocprofv3 --kernel-trace csv: per kernel name, the mean
duration per call (optionally split by call position modulo P)."""
import collections
import csv
import sys


def main(path, top=16):
    r = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for x in r:
        d[x["Kernel_Name"]].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000)
    tot = sum(sum(v) for v in d.values())
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{k[:64]:64s} {len(v):5d} {sum(v)/len(v):9.1f}us {100*sum(v)/tot:6.2f}%")


if __name__ == "__main__":
    main(sys.argv[1])
