#!/usr/bin/env python3
"""Interleaved timing of CSR kernel variants on configs 3 (ragged 16M) and
4 (joint 8M).  Development tool."""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from bench import HipEvents  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    lab = C.CDLL(os.path.join(HERE, "liblab_csr.so"))
    lab.lab_name.restype = C.c_char_p
    lab.lab_launch.argtypes = [C.c_int, C.c_uint64] + [C.c_void_p] * 7
    names = [lab.lab_name(i).decode() for i in range(lab.lab_count())]
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    for kind, G in (("ragged", 1 << 24), ("joint", 1 << 23)):
        grp = batch.CsrGroups.synth(0x5EED0003, kind, G, device=dev)
        ref_c, ref_v = grp.committed_vote()
        slots = int(grp.off[-1].item())
        algo = G * 21 + 8 * slots
        c = torch.empty_like(ref_c)
        v = torch.empty_like(ref_v)
        args = lambda i: (i, G, grp.off.data_ptr(), grp.match.data_ptr(), grp.cfg.data_ptr(),
                          grp.votes.data_ptr(), c.data_ptr(), v.data_ptr(), sp)
        from etcd_amd import _lib
        prod = _lib.load().qb_dev_csr_committed_vote
        if "product" not in names:
            names.append("product")

        def launch(i):
            if names[i] == "product":
                return prod(G, grp.max_slots, grp.off.data_ptr(), grp.match.data_ptr(),
                            grp.cfg.data_ptr(), grp.votes.data_ptr(), c.data_ptr(), v.data_ptr(),
                            sp)
            return lab.lab_launch(*args(i))

        for i, nm in enumerate(names):
            c.zero_()
            launch(i)
            torch.cuda.synchronize()
            if "floor" not in nm:
                ok = torch.equal(c, ref_c) and torch.equal(v, ref_v)
                print(f"check {kind} {nm:22s} {'ok' if ok else 'MISMATCH'}", flush=True)
        ev = HipEvents(2)
        res = {nm: [] for nm in names}
        rng = np.random.default_rng(0)
        for r in range(a.rounds):
            for i in rng.permutation(len(names)):
                launch(int(i))
                ev.record(ev.ev[0], sp)
                for _ in range(a.reps):
                    launch(int(i))
                ev.record(ev.ev[1], sp)
                torch.cuda.synchronize()
                res[names[i]].append(ev.elapsed_ms(0, 1) * 1e3 / a.reps)
        print(f"{kind} G={G} slots/group={slots / G:.2f} algo B/group={algo / G:.1f}")
        for nm in names:
            t = np.median(res[nm])
            print(f"  {nm:22s} {t:8.1f} us  {algo / t / 1e3:7.1f} GB/s  {G / t / 1e3:6.2f} Ggroups/s",
                  flush=True)


if __name__ == "__main__":
    main()
