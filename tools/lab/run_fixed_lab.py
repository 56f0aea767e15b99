#!/usr/bin/env python3
"""Interleaved A/B timing of fixed-layout kernel variants and launch modes
(development tool).  Prints one line per variant: median / min kernel us and
GB/s at 51 algorithmic bytes per group.  Usage (GPU box):
    make -C tools/lab && python tools/lab/run_fixed_lab.py [--groups N]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from bench import HipEvents  # noqa: E402
from etcd_amd import _lib  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipStreamBeginCapture.argtypes = [C.c_void_p, C.c_int]
hip.hipStreamEndCapture.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
hip.hipGraphInstantiate.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_size_t]
hip.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=64)
    ap.add_argument("--focus", default="", help="comma list: interleaved S-stream comparison only")
    ap.add_argument("--streams", type=int, default=2)
    args = ap.parse_args()
    G, B = args.groups, args.batches
    lab = C.CDLL(os.path.join(HERE, "liblab_fixed.so"))
    lab.lab_name.restype = C.c_char_p
    lab.lab_launch.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_void_p, C.c_void_p]
    nv = lab.lab_count()
    names = [lab.lab_name(i).decode() for i in range(nv)]
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    fgs = [batch.FixedGroups.synth(0x5EED0002, 5, G, g_begin=b * G, device=dev) for b in range(B)]
    outs = [(torch.empty(G, dtype=torch.int64, device=dev),
             torch.empty(G, dtype=torch.uint8, device=dev)) for _ in range(B)]
    ref_c, ref_v = fgs[0].committed_vote()
    torch.cuda.synchronize()

    # correctness of compute variants on batch 0
    for i, nm in enumerate(names):
        c, v = outs[0]
        c.zero_()
        v.zero_()
        lab.lab_launch(i, fgs[0].match.data_ptr(), G, fgs[0].voted.data_ptr(),
                       fgs[0].granted.data_ptr(), c.data_ptr(), v.data_ptr(), sp)
        torch.cuda.synchronize()
        if not nm.startswith("floor"):
            ok = torch.equal(c, ref_c) and torch.equal(v, ref_v)
            print(f"check {nm:16s} {'ok' if ok else 'MISMATCH'}")

    if args.focus:
        focus(args, lab, names, fgs, outs, dev, sp)
        return
    L = args.launches
    ev = HipEvents(2 * L)
    times = {nm: [] for nm in names}
    rng = np.random.default_rng(0)
    for r in range(args.rounds):
        order = rng.permutation(nv)
        for i in order:
            for k in range(8):  # warm
                g = fgs[k % B]
                c, v = outs[k % B]
                lab.lab_launch(int(i), g.match.data_ptr(), G, g.voted.data_ptr(),
                               g.granted.data_ptr(), c.data_ptr(), v.data_ptr(), sp)
            for k in range(L):
                g = fgs[k % B]
                c, v = outs[k % B]
                ev.record(ev.ev[2 * k], sp)
                lab.lab_launch(int(i), g.match.data_ptr(), G, g.voted.data_ptr(),
                               g.granted.data_ptr(), c.data_ptr(), v.data_ptr(), sp)
                ev.record(ev.ev[2 * k + 1], sp)
            torch.cuda.synchronize()
            times[names[i]] += [ev.elapsed_ms(2 * k, 2 * k + 1) * 1e3 for k in range(L)]
    bpg = 51
    print(f"G={G} batches={B}  (us per kernel; GB/s at {bpg} B/group)")
    for nm in names:
        t = np.array(times[nm])
        med = np.median(t)
        print(f"{nm:16s} med {med:8.2f}  min {t.min():8.2f}  p90 {np.percentile(t, 90):8.2f}"
              f"  {bpg * G / med / 1e3:8.1f} GB/s")

    # launch modes with the product kernel
    fn = _lib.load().qb_dev_fixed_committed_vote
    argsets = [(5, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(),
                c.data_ptr(), v.data_ptr(), sp) for g, (c, v) in zip(fgs, outs)]
    K = 256
    import time

    def loop(events):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            if events:
                ev2.record(ev2.ev[2 * k], sp)
            fn(*argsets[k % B])
            if events:
                ev2.record(ev2.ev[2 * k + 1], sp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e6

    ev2 = HipEvents(2 * K)
    for _ in range(2):
        a = loop(False)
        b = loop(True)
    kern = np.mean([ev2.elapsed_ms(2 * k, 2 * k + 1) * 1e3 for k in range(K)])
    print(f"launch modes (us/step): loop {a:.2f}  loop+events {b:.2f} (kernel {kern:.2f})",
          flush=True)
    # multi-stream overlap of independent batches, region timing only
    for variant in ("product", "gpt1", "gpt2_nt", "gpt4"):
        vi = names.index(variant) if variant != "product" else -1
        for S in (1, 2, 3, 4):
            streams = [torch.cuda.Stream(dev) for _ in range(S)]
            sps = [s_.cuda_stream for s_ in streams]
            evr = HipEvents(2 + 2 * S)
            best = 1e9
            for rep in range(4):
                torch.cuda.synchronize()
                evr.record(evr.ev[0], sp)
                for j, s_ in enumerate(streams):
                    s_.wait_stream(torch.cuda.current_stream(dev))
                for k in range(K):
                    g = fgs[k % B]
                    c, v = outs[k % B]
                    st = sps[k % S]
                    if vi < 0:
                        fn(5, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(),
                           c.data_ptr(), v.data_ptr(), st)
                    else:
                        lab.lab_launch(vi, g.match.data_ptr(), G, g.voted.data_ptr(),
                                       g.granted.data_ptr(), c.data_ptr(), v.data_ptr(), st)
                for s_ in streams:
                    torch.cuda.current_stream(dev).wait_stream(s_)
                evr.record(evr.ev[1], sp)
                torch.cuda.synchronize()
                best = min(best, evr.elapsed_ms(0, 1) * 1e3 / K)
            print(f"streams {variant:8s} S={S}: {best:7.2f} us/step  "
                  f"{51 * G / best / 1e3:7.1f} GB/s", flush=True)
    # graph capture of K steps with events
    cs = torch.cuda.Stream(dev)
    csp = cs.cuda_stream
    ev3 = HipEvents(2 * K)
    gargs = [(5, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(),
              c.data_ptr(), v.data_ptr(), csp) for g, (c, v) in zip(fgs, outs)]
    torch.cuda.synchronize()
    assert hip.hipStreamBeginCapture(csp, 2) == 0
    for k in range(K):
        ev3.record(ev3.ev[2 * k], csp)
        fn(*gargs[k % B])
        ev3.record(ev3.ev[2 * k + 1], csp)
    graph = C.c_void_p()
    assert hip.hipStreamEndCapture(csp, C.byref(graph)) == 0
    exe = C.c_void_p()
    assert hip.hipGraphInstantiate(C.byref(exe), graph, None, None, 0) == 0
    res = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert hip.hipGraphLaunch(exe, csp) == 0
        cs.synchronize()
        res.append((time.perf_counter() - t0) / K * 1e6)
    try:
        gk = "%.2f" % np.mean([ev3.elapsed_ms(2 * k, 2 * k + 1) * 1e3 for k in range(K)])
    except AssertionError:
        gk = "n/a (event timing unsupported in graphs)"
    print(f"graph+events {min(res):.2f} us/step (kernel {gk})")


def focus(args, lab, names, fgs, outs, dev, sp):
    G, B, S, K = args.groups, args.batches, args.streams, 256
    fn = _lib.load().qb_dev_fixed_committed_vote
    cand = args.focus.split(",")
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    sps = [s_.cuda_stream for s_ in streams]
    evr = HipEvents(2)
    res = {c: [] for c in cand}
    rng = np.random.default_rng(1)
    for r in range(args.rounds):
        for ci in rng.permutation(len(cand)):
            c = cand[ci]
            vi = names.index(c) if c != "product" else -1
            torch.cuda.synchronize()
            evr.record(evr.ev[0], sp)
            for s_ in streams:
                s_.wait_stream(torch.cuda.current_stream(dev))
            for k in range(K):
                g = fgs[k % B]
                o_c, o_v = outs[k % B]
                st = sps[k % S]
                if vi < 0:
                    fn(5, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(),
                       o_c.data_ptr(), o_v.data_ptr(), st)
                else:
                    lab.lab_launch(vi, g.match.data_ptr(), G, g.voted.data_ptr(),
                                   g.granted.data_ptr(), o_c.data_ptr(), o_v.data_ptr(), st)
            for s_ in streams:
                torch.cuda.current_stream(dev).wait_stream(s_)
            evr.record(evr.ev[1], sp)
            torch.cuda.synchronize()
            res[c].append(evr.elapsed_ms(0, 1) * 1e3 / K)
    print(f"focus S={S} G={G} B={B} rounds={args.rounds}")
    for c in cand:
        t = np.array(res[c])
        print(f"{c:14s} med {np.median(t):7.2f} min {t.min():7.2f} max {t.max():7.2f} us/step"
              f"  med {51 * G / np.median(t) / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
