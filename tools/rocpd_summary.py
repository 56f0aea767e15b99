#!/usr/bin/env python3
"""Per-kernel summary (calls, average and total duration) of a rocprofv3
--kernel-trace run stored as its SQLite database (``-o run`` -> run_results.db).
Usage: python tools/rocpd_summary.py <results.db> [name-substring ...]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    want = sys.argv[2:]
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), avg(duration), sum(duration), min(duration), "
                       "max(duration) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[3] for r in rows)
    print(f"{'calls':>7} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_ms':>10} {'pct':>6}  kernel")
    for name, n, avg, s, mn, mx in rows:
        short = name.split("(")[0]
        if want and not any(w in short for w in want):
            continue
        print(f"{n:7d} {avg / 1e3:10.2f} {mn / 1e3:10.2f} {mx / 1e3:10.2f} {s / 1e6:10.3f} "
              f"{100 * s / tot:6.2f}  {short}")


if __name__ == "__main__":
    main()
