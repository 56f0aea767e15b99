#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes of the bench command.

Recipe (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  pass 1: rocprofv3 --pmc FETCH_SIZE --output-format csv -d D1 -o run -- python3 bench.py ...
  pass 2: rocprofv3 --pmc WRITE_SIZE --output-format csv -d D2 -o run -- python3 bench.py ...
(separate passes: FETCH_SIZE uses 3 of the 4 TCC slots, WRITE_SIZE 2).
Counter values are KiB.  gfx950 correction: FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced streaming read, so the read side
is doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.  The narrow
(2 B/lane) mask loads and vote stores are a small uncalibrated share (4 of the
51 bytes per group) and are treated like the wide ones.

Only the timed HBM-rotating dispatches are used: dispatches [W, W+K) of the
kernel in launch order.

    python tools/pmc_traffic.py --fetch D1/run_counter_collection.csv \
        --write D2/run_counter_collection.csv --kernel k_fixed --warmup 5 --steps 50 \
        --key fixed_n5_G1048576 --algo-bytes 53477376 --out profiles/pmc_traffic.json
"""
import argparse
import csv
import json
import os

import numpy as np


def base_name(full: str) -> str:
    """A kernel's unqualified name without template arguments or parameters:
    "void qb::bk::k_csr_apply<12, 8, false>(...)" -> "k_csr_apply"."""
    s = full[5:] if full.startswith("void ") else full
    s = s.replace("(anonymous namespace)::", "")
    for ch in "<(":
        i = s.find(ch)
        if i >= 0:
            s = s[:i]
    return s.rsplit("::", 1)[-1].strip()


def per_dispatch(path, kernel, counter):
    """Per-dispatch counter values of the kernels whose base name is exactly
    ``kernel`` (round 3 matched substrings, so "k_csr_apply" also took
    k_csr_apply_deferred's dispatches into its median)."""
    vals = {}
    for r in csv.DictReader(open(path)):
        if base_name(r.get("Kernel_Name", "")) != kernel:
            continue
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_fixed",
                    help="kernel name substring; a comma-separated list sums the medians of "
                         "every listed kernel (a multi-kernel step, one dispatch of each per step)")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--from-end", action="store_true",
                    help="take each kernel's LAST --steps dispatches (the tracker bench runs nothing "
                         "after its region, and its setup dispatches some step kernels once more "
                         "than the others, which shifts a [W, W+K) window per kernel)")
    ap.add_argument("--key", required=True)
    ap.add_argument("--algo-bytes", type=float, required=True, help="algorithmic bytes/launch")
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default=None,
                    help="where the two CSVs are committed (profiles/rNN/...), stored in the entry")
    a = ap.parse_args()
    fk = wk = 0.0
    per = {}
    for kern in a.kernel.split(","):
        f = per_dispatch(a.fetch, kern, "FETCH_SIZE")
        w = per_dispatch(a.write, kern, "WRITE_SIZE")
        if a.from_end:
            f, w = f[-a.steps:], w[-a.steps:]
        else:
            f, w = f[a.warmup:a.warmup + a.steps], w[a.warmup:a.warmup + a.steps]
        if not f or not w:
            raise SystemExit(f"no matching dispatches for {kern}")
        per[kern] = {"read_bytes_corrected": 2.0 * float(np.median(f)) * 1024.0,
                     "write_bytes": float(np.median(w)) * 1024.0}
        fk += float(np.median(f))
        wk += float(np.median(w))
    read_b = 2.0 * fk * 1024.0   # gfx950 FETCH_SIZE x2 correction
    write_b = wk * 1024.0
    rec = {
        "kernel": a.kernel, "dispatches": len(f), "per_kernel": per,
        "fetch_size_kib_median_raw": fk, "write_size_kib_median": wk,
        "read_bytes_corrected": read_b, "write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": a.algo_bytes,
        "traffic_over_algorithmic": (read_b + write_b) / a.algo_bytes,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                  "FETCH_SIZE x2 (gfx950 wide-read correction); KiB->bytes x1024; kernels "
                  "matched by exact base name; " + ("last K dispatches of each kernel"
                                                   if a.from_end else "dispatches [W, W+K)"),
    }
    if a.source:
        rec["source"] = a.source
    doc = {}
    if os.path.exists(a.out):
        doc = json.load(open(a.out))
    doc[a.key] = rec
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
