#!/usr/bin/env python3
"""Interleaved A/B of qb_dev_csr_committed_vote between the in-tree library
and another build (tools/lab/old/libquorumbatch.so) on configs 3 and 4, with a
bit-exactness check between them.  Development tool."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from bench import HipEvents  # noqa: E402
from etcd_amd import _lib  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402


def main():
    new = _lib.load()
    old = C.CDLL(os.path.join(HERE, "old", "libquorumbatch.so"))
    old.qb_dev_csr_committed_vote.argtypes = new.qb_dev_csr_committed_vote.argtypes
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    for kind, G in (("ragged", 1 << 24), ("joint", 1 << 23)):
        grp = batch.CsrGroups.synth(0x5EED0003 if kind == "ragged" else 0x5EED0004, kind, G,
                                    device=dev)
        outs = {}
        for nm, lib in (("old", old), ("new", new)):
            c = torch.empty(G, dtype=torch.int64, device=dev)
            v = torch.empty(G, dtype=torch.uint8, device=dev)
            outs[nm] = (lib, c, v)
        call = lambda nm: outs[nm][0].qb_dev_csr_committed_vote(
            G, grp.max_slots, grp.off.data_ptr(), grp.match.data_ptr(), grp.cfg.data_ptr(),
            grp.votes.data_ptr(), outs[nm][1].data_ptr(), outs[nm][2].data_ptr(), sp)
        for nm in outs:
            call(nm)
        torch.cuda.synchronize()
        same = torch.equal(outs["old"][1], outs["new"][1]) and torch.equal(outs["old"][2], outs["new"][2])
        ev = HipEvents(2)
        res = {nm: [] for nm in outs}
        for r in range(9):
            for nm in (("old", "new") if r % 2 else ("new", "old")):
                call(nm)
                ev.record(ev.ev[0], sp)
                for _ in range(10):
                    call(nm)
                ev.record(ev.ev[1], sp)
                torch.cuda.synchronize()
                res[nm].append(ev.elapsed_ms(0, 1) * 100)
        print(kind, "bit-identical" if same else "MISMATCH",
              {nm: round(float(np.median(t)), 1) for nm, t in res.items()}, "us", flush=True)


if __name__ == "__main__":
    main()
