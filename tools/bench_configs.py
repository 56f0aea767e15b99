#!/usr/bin/env python3
"""Throughput of every BASELINE config on one GPU (bench.py measures only
configs[1]; these are the parity-test configs, measured the same way).

  config 1  plumbing: BenchmarkMajorityConfig_CommittedIndex (bench_test.go:24-40),
            voters 1..11, CPU ns/op beside GPU ns per group
  config 3  16M groups ragged 3-9 voters + 0-2 learners (CSR)
  config 4  joint 5+5 (overlap 0-5), 8M groups = one GPU's shard of 64M
  config 5  streaming tracker: 16M 5-voter groups, one MsgAppResp per group
            per step on average (1% stale term), apply + commit advance

Prints one JSON line per config: groups/s (group-steps/s for config 5),
per-launch device time (HIP events around R back-to-back launches / R),
algorithmic GB/s and fraction of the 8 TB/s HBM peak.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import HBM_PEAK_GBS, HipEvents  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402

dev = torch.device("cuda", 0)


GPU_ONLY = False  # the command line's --gpu-only (functions take gpu_only= explicitly too)


def time_region(fn, reps, warm_s=0.3, regions=5):
    """Per-call device time: median over `regions` event-timed regions of
    `reps` back-to-back calls, after ~warm_s seconds of warm-up calls (a
    fresh box needs that long before its clocks settle: with 3 warm-up
    calls the first config measured up to 20 % slow)."""
    import time
    sp = torch.cuda.current_stream(dev).cuda_stream
    t0 = time.perf_counter()
    while True:
        fn()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= warm_s:
            break
    ev = HipEvents(2)
    ts = []
    for _ in range(regions):
        torch.cuda.synchronize()
        ev.record(ev.ev[0], sp)
        for _ in range(reps):
            fn()
        ev.record(ev.ev[1], sp)
        torch.cuda.synchronize()
        ts.append(ev.elapsed_ms(0, 1) / 1e3 / reps)
    ev.close()
    return float(np.median(ts))


def cpu_rate(fn, groups, seconds=2.0):
    """groups/s of a CPU oracle call repeated for ~seconds."""
    import time
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps * groups / dt


def report(name, groups, t, algo_bytes, extra=None):
    gbs = algo_bytes / t / 1e9
    d = {"config": name, "groups_per_s": groups / t, "per_launch_us": t * 1e6,
         "algo_bytes_per_launch": algo_bytes, "algo_bytes_per_group": algo_bytes / groups,
         "achieved_GBs": gbs, "frac_hbm_peak": gbs / HBM_PEAK_GBS}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def plumbing_config(reps):
    """BASELINE configs[0]: BenchmarkMajorityConfig_CommittedIndex
    (quorum/bench_test.go:24-40), voters in {1,3,5,7,9,11}.  CPU: the
    faithful C restatement (map config + map AckedIndexer + insertion sort),
    one config called in a loop on 1 thread, ns/op.  GPU beside it: the same
    CommittedIndex over 16M groups of that width in one launch (fixed layout,
    CommittedIndex only), device ns per group."""
    import time
    from tests import oracle_c as oc
    lib = oc.load()
    G = 1 << 24
    for n in (1, 3, 5, 7, 9, 11):
        iters, t = 1 << 20, 0.0
        while True:
            t0 = time.perf_counter()
            lib.orc_bench_plumbing(n, iters, 0x5EED0001)
            t = time.perf_counter() - t0
            if t >= 0.5:
                break
            iters *= 4
        fg = batch.FixedGroups.synth(0x5EED0001, n, G, device=dev)
        c = torch.empty(G, dtype=torch.int64, device=dev)
        tg = time_region(lambda: fg.committed_vote(c, want_vote=False), reps)
        print(json.dumps({"config": f"plumbing voters={n}", "cpu_ns_per_op": t / iters * 1e9,
                          "cpu_kind": "port (faithful C restatement of majority.go, 1 thread)",
                          "gpu_ns_per_group": tg / G * 1e9, "gpu_groups_per_launch": G,
                          "gpu_achieved_GBs": G * (8 * n + 8) / tg / 1e9}), flush=True)
        del fg, c


def csr_config(kind, G, reps, *, reporter=None, gpu_only=None):
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    grp = batch.CsrGroups.synth(0x5EED0003 if kind == "ragged" else 0x5EED0004, kind, G,
                                device=dev)
    slots = int(grp.off[-1].item())
    c = torch.empty(G, dtype=torch.int64, device=dev)
    v = torch.empty(G, dtype=torch.uint8, device=dev)
    t = time_region(lambda: grp.committed_vote(c, v), reps)
    # off (4) + cfg (4) + votes (4) + match (8 s) + commit (8) + vote (1)
    algo = G * (4 + 4 + 4 + 8 + 1) + 8 * slots + 4
    if gpu_only:
        reporter(f"{kind} CSR", G, t, algo, {"mean_slots": slots / G})
        return
    # CPU beside it: the oracle's SoA C restatement on a bounded sample
    from tests import oracle_c as oc
    threads = max(1, min(16, os.cpu_count() or 1))
    Gs = 1 << 20
    off, m, cfg, votes = oc.gen_csr(0x5EED0003 if kind == "ragged" else 0x5EED0004, kind, Gs)
    cpu = cpu_rate(lambda: oc.csr_eval(off, m, cfg, votes, threads=threads), Gs)
    cpu1 = cpu_rate(lambda: oc.csr_eval(off, m, cfg, votes), Gs)
    reporter(f"{kind} CSR", G, t, algo, {"mean_slots": slots / G,
           "cpu_baseline": {"value": cpu, "unit": "groups/s", "cores": threads, "kind": "port",
                            "value_1thread": cpu1,
                            "sample": f"{Gs} groups, C SoA restatement (oracle)"}})


def tracker_config(G, reps, seed=55, E=64, warm_steps=4, regions=5, *, reporter=None,
                   gpu_only=None):
    """Config 5: streaming MsgAppResp batches.  The leader holds E new
    entries per step (its own match, slot 0, is already at the last one);
    batch k acknowledges index last + (k+1)·E − lag (lag < 96) for a random
    follower of a random group, 1 % stale-term — so every step raises
    matches and advances commits, as a live stream does (the same batch
    replayed would leave the state unchanged after its first application).
    Each timed region restores the start state (untimed), runs warm_steps
    batches, then times `reps` further distinct batches; median of regions."""
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    n = 5
    rng = np.random.default_rng(seed)
    tr = batch.FixedTracker(n, G, dev)
    fg = batch.FixedGroups.synth(0x5EED0005, n, G, device=dev, with_term_start=True)
    tr.match.copy_(fg.match)
    tr.term_start.copy_(fg.term_start)
    tr.term.fill_(7)
    tr.commit_advance()
    last = fg.match[0].clone()
    del fg
    nb = warm_steps + reps
    tr.match[0].copy_(last + nb * E)  # the leader's own match (raft.go:747-748 appendEntry)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    batches = []
    for k in range(nb):
        group = torch.randint(0, G, (G,), generator=gen, device=dev, dtype=torch.int32)
        slot = torch.randint(1, n, (G,), generator=gen, device=dev, dtype=torch.int32)
        lag = torch.randint(0, 96, (G,), generator=gen, device=dev, dtype=torch.int64)
        index = last[group.long()] + (k + 1) * E - lag
        term = torch.where(torch.rand(G, generator=gen, device=dev) < 0.01, 6, 7).to(torch.int64)
        batches.append(batch.AppRespBatch(group, slot.to(torch.uint8), index, term))
    snap = {k_: getattr(tr, k_).clone() for k_ in ("match", "committed", "active", "stepdown_at")}
    sp = torch.cuda.current_stream(dev).cuda_stream

    def restore():
        for k_, v_ in snap.items():
            getattr(tr, k_).copy_(v_)

    def stream_time(step):
        ev = HipEvents(2)
        ts = []
        for r in range(regions + 1):  # region 0 warms the clocks, not reported
            restore()
            for k in range(warm_steps):
                step(batches[k])
            torch.cuda.synchronize()
            ev.record(ev.ev[0], sp)
            for k in range(warm_steps, nb):
                step(batches[k])
            ev.record(ev.ev[1], sp)
            torch.cuda.synchronize()
            if r:
                ts.append(ev.elapsed_ms(0, 1) / 1e3 / reps)
        ev.close()
        return float(np.median(ts))

    def two_call(b):
        tr.apply_appresp(b)
        tr.commit_advance()

    t_two = t_apply = t_commit = float("nan")
    if not gpu_only:  # A/B runs time the bucketed step alone
        t_two = stream_time(two_call)
        t_apply = stream_time(lambda b: tr.apply_appresp(b))
        t_commit = time_region(lambda: tr.commit_advance(), reps)
    t = stream_time(lambda b: tr.step(b))
    adv = torch.zeros(G, dtype=torch.uint8, device=dev)
    restore()
    for k in range(nb - 1):
        tr.step(batches[k])
    tr.step(batches[nb - 1], adv)
    advanced_last = int(adv.sum().item())
    applied_last = tr.stats_dict()["applied"]
    del batches
    # record 21 B + match RMW 16 B per message; commit advance
    # reads match 40 + term_start 8 + committed 8, writes committed 8 per group
    algo = G * (21 + 16) + G * 64
    # CPU beside it: the sequential one-record-at-a-time oracle (the Go
    # stepLeader loop restated) on a bounded sample, 1 thread
    if gpu_only:
        reporter("streaming tracker (bucketed step)", G, t, algo, {"unit": "group-steps/s"})
        return
    from tests import oracle_c as oc
    Gs = 1 << 20
    m0, _, _, ts0 = oc.gen_fixed(0x5EED0005, n, Gs)
    st = {"match": m0, "active": np.zeros(Gs, np.uint16), "term": np.full(Gs, 7, np.uint64),
          "term_start": ts0, "committed": np.zeros(Gs, np.uint64),
          "stepped_down": np.zeros(Gs, np.uint8)}
    oc.commit_all(n, st["match"], ts0, st["committed"])
    grp_ = rng.integers(0, Gs, size=Gs).astype(np.uint32)
    flg = rng.integers(1, n, size=Gs).astype(np.uint8)
    lag = rng.integers(0, 96, size=Gs).astype(np.uint64)
    lst = m0[0][grp_]
    idx = np.where(lag < lst, lst - lag, np.uint64(0))
    trm = np.where(rng.random(Gs) < 0.01, 6, 7).astype(np.uint64)
    cpu1 = cpu_rate(lambda: oc.appresp_sequential(n, Gs, (grp_, flg, idx, trm), st), Gs)
    reporter("streaming tracker (bucketed step)", G, t, algo,
           {"two_call_us": t_two * 1e6, "atomic_apply_us": t_apply * 1e6,
            "workload": f"{G} groups x 5 voters, {G} records per step (streaming: {E} new "
                        f"entries per step), 1% stale-term; last step: {applied_last} applied, "
                        f"{advanced_last} commits advanced",
            "commit_advance_us": t_commit * 1e6, "unit": "group-steps/s",
            "cpu_baseline": {"value": cpu1, "unit": "group-steps/s", "cores": 1, "kind": "port",
                             "sample": f"{Gs} records on {Gs} groups, sequential C restatement"}})


def wire_tracker_tick(G, nb, E=64, seed=77, dev_=None):
    """The composed per-tick workload (VERDICT r4 Missing 3): G 5-voter groups
    (FIXED layout, leader term 20007 since B = 2^35), nb ticks of G MsgAppResp
    each, encoded as gogoproto bytes on the device (wire.encode_appresp), from
    a random follower of a random group, 1 % stale-term (20006); tick k acks
    last + (k+1)·E − lag.  Returns (tracker, snapshot, ticks, rows, off, ids):
    tick = (buf, nbytes, msg_off, msg_group, direct AppRespBatch)."""
    from etcd_amd.quorum import wire
    d = dev_ or dev
    n = 5
    B = 1 << 35
    gen = torch.Generator(device=d)
    gen.manual_seed(seed)
    tr = batch.FixedTracker(n, G, d)
    last = B + 1024 + torch.randint(0, 1 << 20, (G,), generator=gen, device=d, dtype=torch.int64)
    tr.match[0].copy_(last + nb * E)  # the leader's own match (raft.go:747-748 appendEntry)
    for s_ in range(1, n):
        tr.match[s_].copy_(last - torch.randint(0, 200, (G,), generator=gen, device=d,
                                                dtype=torch.int64))
    tr.term.fill_(20007)
    tr.term_start.fill_(B)
    tr.commit_advance()
    off = torch.arange(0, n * G + 1, n, dtype=torch.int32, device=d)
    gg = torch.arange(G, dtype=torch.int64, device=d)
    ids = (16384 + torch.arange(n, dtype=torch.int64, device=d)[None, :] * 200000
           + (gg % 100000)[:, None]).reshape(-1)  # ascending per group
    rows = wire.group_rows(off, ids)
    ticks = []
    for k in range(nb):
        group = torch.randint(0, G, (G,), generator=gen, device=d, dtype=torch.int64)
        slot = torch.randint(1, n, (G,), generator=gen, device=d, dtype=torch.int64)
        lag = torch.randint(0, 96, (G,), generator=gen, device=d, dtype=torch.int64)
        index = last[group] + (k + 1) * E - lag
        term = torch.where(torch.rand(G, generator=gen, device=d) < 0.01, 20006, 20007)
        to = ids[group * n]
        frm = ids[group * n + slot]
        rej = torch.zeros(G, dtype=torch.bool, device=d)
        buf, nbytes, moff = wire.encode_appresp(to, frm, term, index, rej)
        direct = batch.AppRespBatch(group.to(torch.int32), slot.to(torch.uint8), index,
                                    term.to(torch.int64))
        ticks.append((buf, nbytes, moff, group.to(torch.int32), direct))
    snap = {k_: getattr(tr, k_).clone() for k_ in ("match", "committed", "active", "stepdown_at")}
    return tr, snap, ticks, rows, off, ids


def wire_tracker_csr_tick(G, nb, E=64, seed=79, dev_=None):
    """The composed workload over the CSR tracker (configs[2]'s ragged groups:
    3-9 voters + 0-2 learners, BASELINE configs[4]'s streaming step): G groups,
    nb ticks of G device-encoded MsgAppResp from a random non-leader slot of a
    random group, leader term 20007 (1 % stale 20006), indexes past 2^35 (6-byte
    varints); slot IDs ascending per group (3-byte varints).  Returns (tracker,
    snapshot, ticks, rows, off, ids) as wire_tracker_tick."""
    import bench
    from etcd_amd.quorum import wire
    d = dev_ or dev
    B = 1 << 35
    grp = batch.CsrGroups.synth(bench.CSR_SEED["ragged"], "ragged", G, device=d)
    tr = batch.CsrTracker(grp.off, grp.cfg, max_slots=grp.max_slots, device=d)
    del grp
    gen = torch.Generator(device=d)
    gen.manual_seed(seed)
    sizes = (tr.off[1:] - tr.off[:-1]).long()
    first = tr.off[:-1].long()
    gidx = torch.repeat_interleave(torch.arange(G, device=d), sizes)
    # the leader (slot 0) at last, followers up to 200 behind (6-byte varints)
    last = B + 1024 + torch.randint(0, 1 << 20, (G,), generator=gen, device=d, dtype=torch.int64)
    tr.match.copy_(last[gidx] - torch.randint(0, 200, (tr.S,), generator=gen, device=d,
                                              dtype=torch.int64))
    tr.match[first] = last
    tr.term.fill_(20007)
    tr.term_start.copy_(last - 64)
    tr.commit_advance()
    sl = torch.arange(tr.S, device=d) - first[gidx]
    ids = 16384 + sl * 100000 + (gidx % 100000)  # ascending per group
    rows = wire.group_rows(tr.off, ids)
    ticks = []
    for k in range(nb):
        group = torch.randint(0, G, (G,), generator=gen, device=d, dtype=torch.int64)
        r_ = torch.randint(0, 1 << 30, (G,), generator=gen, device=d, dtype=torch.int64)
        slot = 1 + r_ % (sizes[group] - 1)
        lag = torch.randint(0, 96, (G,), generator=gen, device=d, dtype=torch.int64)
        index = last[group] + (k + 1) * E - lag
        term = torch.where(torch.rand(G, generator=gen, device=d) < 0.01, 20006, 20007)
        rej = torch.zeros(G, dtype=torch.bool, device=d)
        buf, nbytes, moff = wire.encode_appresp(ids[first[group]], ids[first[group] + slot], term,
                                                index, rej)
        direct = batch.AppRespBatch(group.to(torch.int32), slot.to(torch.uint8), index,
                                    term.to(torch.int64))
        ticks.append((buf, nbytes, moff, group.to(torch.int32), direct))
    tr.match[first] = last + nb * E  # the leader appended nb * E entries
    snap = {k_: getattr(tr, k_).clone() for k_ in ("match", "committed", "active", "stepdown_at")}
    return tr, snap, ticks, rows, tr.off, ids


def wire_tracker_config(G, reps, warm=4, regions=3, *, reporter=None, gpu_only=None,
                        fused_only=False, csr=False):
    """Composed row: wire bytes -> tracker tick, per tick (rafthttp/stream.go:466
    decode -> raft.go:1106-1259 stepLeader MsgAppResp -> maybeCommit), G
    groups and G messages per tick, in one call (round 6:
    qb_dev_ingest_fixed_tracker_step — the decoder writes the tracker step's
    level-1 buckets, no record columns between them); beside it the chain of
    round 5 (qb_dev_ingest_messages_rows -> records -> qb_dev_fixed_tracker_step)
    and its two halves.  Parity in the row (size-independent): every status
    OK and the tracker state after the ticks through the one call equals the
    state the direct step (same columns, no wire) reaches, and so does the
    chain's (its decoded columns equal the encoded ones) — bit-exact.  The GPU
    suite checks both against the C oracles (tests/test_gpu_wire.py,
    tests/test_gpu_wire_tracker.py)."""
    reporter = reporter or report
    from etcd_amd.quorum import wire
    nb = warm + reps
    tr, snap, ticks, rows, off, ids = (wire_tracker_csr_tick if csr else wire_tracker_tick)(G, nb)
    sp = torch.cuda.current_stream(dev).cuda_stream

    def restore():
        for k_, v_ in snap.items():
            getattr(tr, k_).copy_(v_)

    def chain(tk):
        ib, _, _ = wire.ingest(tk[0], tk[1], tk[2], tk[3], off, ids, rows=rows)
        tr.step(batch.AppRespBatch(ib.group, ib.flags, ib.index, ib.term))

    def fused(tk):
        wire.ingest_tracker_step(tr, tk[0], tk[1], tk[2], tk[3], rows=rows, ids=ids)

    def timed(fn):
        ev = HipEvents(2)
        ts = []
        for r in range(regions + 1):
            restore()
            for k in range(warm):
                fn(ticks[k])
            torch.cuda.synchronize()
            ev.record(ev.ev[0], sp)
            for k in range(warm, nb):
                fn(ticks[k])
            ev.record(ev.ev[1], sp)
            torch.cuda.synchronize()
            if r:
                ts.append(ev.elapsed_ms(0, 1) / 1e3 / reps)
        ev.close()
        return float(np.median(ts))
    t = timed(fused)
    if fused_only:  # development A/B: the one call alone
        t_chain = t_ingest = t_step = float("nan")
    else:
        t_chain = timed(chain)
        t_ingest = timed(lambda tk: wire.ingest(tk[0], tk[1], tk[2], tk[3], off, ids, rows=rows))
        t_step = timed(lambda tk: tr.step(tk[4]))
    # parity: the one call and the chain against the direct step over every tick
    bad = 0
    restore()
    for tk in ticks:
        status = wire.ingest_tracker_step(tr, tk[0], tk[1], tk[2], tk[3], rows=rows, ids=ids)
        bad += int((status != 0).sum())
    via_fused = {k_: getattr(tr, k_).clone() for k_ in snap}
    restore()
    for tk in ticks:
        ib, status, _ = wire.ingest(tk[0], tk[1], tk[2], tk[3], off, ids, rows=rows)
        d = tk[4]
        bad += int((status != 0).sum()) + int((ib.group != d.group).sum())
        bad += int((ib.flags != d.flags).sum()) + int((ib.index != d.index).sum())
        bad += int((ib.term != d.term).sum())
        tr.step(batch.AppRespBatch(ib.group, ib.flags, ib.index, ib.term))
    via_wire = {k_: getattr(tr, k_).clone() for k_ in snap}
    restore()
    for tk in ticks:
        tr.step(tk[4])
    for k_ in snap:
        bad += int((getattr(tr, k_) != via_wire[k_]).sum())
        bad += int((getattr(tr, k_) != via_fused[k_]).sum())
    nbytes = ticks[0][1]
    del ticks
    # algorithmic bytes per message: its wire bytes, msg_off 8, envelope group
    # 4, the group's slot IDs 40 (wire row), its status byte 1; the tracker's
    # match RMW 16 and the commit advance 64 per group (configs[4] row) — the
    # decoded records are intermediate, not algorithmic
    if csr:  # the CSR step's row (configs[4] CSR: 117 B per group-step; slot IDs 8 B each)
        sl = float((off[-1].item()) / G)
        algo = nbytes + G * (8 + 4 + 8 * sl + 1) + G * (117 - 21)
    else:
        algo = nbytes + G * (8 + 4 + 40 + 1) + G * (16 + 64)
    reporter("wire -> tracker-csr tick (composed)" if csr else "wire -> tracker tick (composed)",
             G, t, algo,
             {"unit": "group-steps/s",
              "form": "one call (qb_dev_ingest_%s_tracker_step)" % ("csr" if csr else "fixed"),
              "chain_us": t_chain * 1e6, "chain_ingest_us": t_ingest * 1e6,
              "chain_tracker_step_us": t_step * 1e6,
              "bytes_per_message": nbytes / G,
              "parity": "bit-exact" if bad == 0 else f"MISMATCH {bad}",
              "parity_check": f"{nb} ticks of {G} messages: every status OK; tracker state "
                              "(match, committed, active, stepdown_at) through the one call == "
                              "through the chain == the direct step's; the chain's decoded "
                              "columns == the encoded columns"})
    if bad:
        raise AssertionError(f"wire -> tracker tick: {bad} mismatches")


def leader_row_parity(kind, Gs=1 << 18):
    """The row's own parity (bench next_rows): the same workload generator at
    Gs groups through both entry points (the group-ordered array and the
    outbox), every state array, message, step-down entry and group flag
    against the C oracle (oracle/leader_oracle.c, the stepLeader loop one
    record at a time); the streaming leader for two consecutive batches.
    Returns "bit-exact" or the mismatching fields."""
    from etcd_amd.quorum.leader import (readindex_inbox, streaming_inbox, synth_readindex,
                                        synth_streaming)
    from tests import oracle_c as oc
    bad = []
    forms = (False, True, "read_states") if kind == "readindex" else (False, True)
    for outbox in forms:
        name = {False: "ordered", True: "outbox", "read_states": "outbox+read_states"}[outbox]
        if kind == "leader":
            lg, base = synth_streaming(Gs, device=dev)
            inboxes = [streaming_inbox(Gs, base, k, device=dev) for k in range(2)]
            Q, cap = 0, 6 * Gs
        else:
            lg, last_ctx, _ = synth_readindex(Gs, 4, device=dev)
            inboxes = [readindex_inbox(Gs, last_ctx, device=dev)]
            Q, cap = 4, 8 * Gs
        host = {k: v.copy() for k, v in lg.numpy().items()}
        for k, ib in enumerate(inboxes):
            if outbox == "read_states":
                res = lg.step_outbox(ib, read_states=True)
            else:
                res = lg.step_outbox(ib) if outbox else lg.step(ib, msg_cap=cap)
            rec = {"group": ib.group.cpu().numpy().view(np.uint32), "flags": ib.flags.cpu().numpy(),
                   "index": ib.index.cpu().numpy().view(np.uint64),
                   "term": ib.term.cpu().numpy().view(np.uint64),
                   "hint": ib.hint.cpu().numpy().view(np.uint64),
                   "log_term": ib.log_term.cpu().numpy().view(np.uint64)}
            msgs, total, sd, gf, _ = oc.leader_step(host, lg.inflight_cap, Q, 0, rec, threads=16,
                                                    msg_cap=cap)
            dev_state = lg.numpy()
            bad += [f"{name} step {k}: {n}" for n in host
                    if not np.array_equal(dev_state[n], host[n])]
            if outbox == "read_states":  # the local answers as ReadStates, the rest as messages
                local = msgs["type"] == 255
                roff = np.zeros(Gs + 1, np.int64)
                roff[1:] = np.cumsum(np.bincount(msgs["group"][local], minlength=Gs))
                if not (local.any() and total == len(msgs)
                        and np.array_equal(res.read_states["index"], msgs["index"][local])
                        and np.array_equal(res.read_states["ctx"], msgs["aux"][local])
                        and np.array_equal(res.read_off, roff)):
                    bad.append(f"{name} step {k}: read states")
                msgs = msgs[~local]
                total = len(msgs)
            if res.msg_total != total or not np.array_equal(res.msgs.view(np.uint8),
                                                            msgs.view(np.uint8)):
                bad.append(f"{name} step {k}: messages")
            if not (np.array_equal(res.stepdown_at, sd) and np.array_equal(res.gflags, gf)):
                bad.append(f"{name} step {k}: stepdown / flags")
        del lg
    torch.cuda.empty_cache()
    return "bit-exact" if not bad else "MISMATCH " + "; ".join(bad[:6])


def leader_config(G, reps, warm=4, shuffle=True, *, reporter=None, gpu_only=None):
    """§8f rows 1-2: the leader inbox step (qb_dev_leader_step) on streaming
    MsgAppResp batches (one per group per step), group-steps/s."""
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    from etcd_amd.quorum.leader import synth_streaming, streaming_inbox
    lg, base = synth_streaming(G, device=dev)
    steps = warm + reps
    inboxes = [streaming_inbox(G, base, k, device=dev, shuffle=shuffle) for k in range(steps)]
    stats = torch.zeros(8, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    snap = {k: v.clone() for k, v in lg.t.items()}

    def timed(step):
        # the same start state and the same `steps` batches for each form
        for k_, v_ in snap.items():
            lg.t[k_].copy_(v_)
        for k in range(warm):
            step(inboxes[k])
        torch.cuda.synchronize()
        stats.zero_()
        ev = HipEvents(2)
        ev.record(ev.ev[0], sp)
        for k in range(warm, steps):
            step(inboxes[k])
        ev.record(ev.ev[1], sp)
        torch.cuda.synchronize()
        dt = ev.elapsed_ms(0, 1) / 1e3 / reps
        ev.close()
        return dt, stats.cpu().tolist()
    # the group-ordered array (qb_dev_leader_step: step, scan, copy) and the
    # per-group outbox the step writes (qb_dev_leader_step_outbox)
    t_ord, st = timed(lambda ib: lg.step(ib, msg_cap=6 * G, stats=stats, fetch=False))
    t, st_ob = timed(lambda ib: lg.step_outbox(ib, stats=stats, fetch=False))
    assert st_ob[6] == st[6], "outbox and ordered forms generated different message counts"
    msgs = st[6] / reps
    # per group-step: record 21 B; group state read 84 B (off 4, cfg 4, meta 4,
    # term/committed/first/last/snap/snap_term/max_ents 56, run 16) + commit
    # and meta written 12 B; 5 slots x (match, next, psnap 24 + pstate 1 +
    # infl_pos 4) read 145 B; the acking follower's freed window entry 8 B and
    # match/next/pstate/infl_pos written 21 B; the record grouping's scan 8 B
    # per group; messages: the outbox form writes each 40 B message once and
    # a 4 B count per group; the ordered form stores, re-reads and writes
    # each (40 B x 3) and scans the counts (8 B per group).
    base = G * (21 + 84 + 12 + 145 + 8 + 21 + 8)
    algo = base + G * 4 + msgs * 40
    algo_ord = base + G * 8 + msgs * 40 * 3
    ordered = {"ordered_us": t_ord * 1e6, "ordered_algo_bytes": algo_ord,
               "ordered_frac": algo_ord / t_ord / 1e9 / HBM_PEAK_GBS,
               "form": "qb_dev_leader_step_outbox (per-group outbox); ordered_* = "
                       "qb_dev_leader_step (group-ordered array)"}
    if not shuffle or gpu_only:
        extra = {"unit": "group-steps/s", "msgs_per_step": msgs, **ordered}
        if shuffle and reporter is not report:  # the default run's next_rows: the row's own parity
            extra["parity"] = leader_row_parity("leader")
            extra["parity_check"] = ("the same stream at 256K groups, two batches, ordered and "
                                     "outbox forms vs the C oracle: state, messages, step-downs")
        reporter("leader inbox step" + ("" if shuffle else ", records in group order (lab)"), G, t,
                 algo, extra)
        return
    # CPU beside it: the C restatement (oracle/leader_oracle.c, the Go
    # stepLeader loop one record at a time) on a bounded sample of the same
    # workload, 16 threads (groups partitioned) and 1 thread.
    import time
    from tests import oracle_c as oc
    Gs = 1 << 20
    lgc, basec = synth_streaming(Gs, device="cpu")
    cpu = {}
    for threads in (16, 1):
        host = {k: v.copy() for k, v in lgc.numpy().items()}
        t0 = time.perf_counter()
        n_steps = 0
        while True:
            ib = streaming_inbox(Gs, basec, n_steps, device="cpu")
            rec = {"group": ib.group.numpy().view(np.uint32), "flags": ib.flags.numpy(),
                   "index": ib.index.numpy().view(np.uint64),
                   "term": ib.term.numpy().view(np.uint64),
                   "hint": ib.hint.numpy().view(np.uint64),
                   "log_term": ib.log_term.numpy().view(np.uint64)}
            t1 = time.perf_counter()
            oc.leader_step(host, 32, 0, 0, rec, threads=threads, msg_cap=6 * Gs)
            n_steps += 1
            cpu.setdefault(threads, 0.0)
            cpu[threads] += time.perf_counter() - t1
            if time.perf_counter() - t0 > 6 or n_steps >= 24:
                break
        cpu[threads] = n_steps * Gs / cpu[threads]
    reporter("leader inbox step (streaming MsgAppResp)", G, t, algo,
           {"unit": "group-steps/s", "msgs_per_step": msgs,
            "applied_per_step": st[0] / reps, "inflight_cap": 32, "voters": 5,
            "cpu_baseline": {"value": cpu[16], "unit": "group-steps/s", "cores": 16,
                             "kind": "port", "value_1thread": cpu[1],
                             "sample": f"{Gs} groups x consecutive steps of the same workload, "
                                       "C restatement of stepLeader (oracle/leader_oracle.c)"}})


def wire_config(M, reps, G=None, rows=False, *, reporter=None, gpu_only=None):
    """§8f row 3: wire ingest of M gogoproto-encoded responses (MsgAppResp +
    10% MsgHeartbeatResp with read contexts) to M/4 5-voter leaders (G given:
    a development variant with a small, cache-resident group table)."""
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    from etcd_amd.quorum import wire
    from tests import oracle_c as oc
    G = G or M // 4
    buf, moff, grp, off, ids = wire.synth_response_stream(M, G)
    d_buf = torch.from_numpy(buf).to(dev)
    d_moff = torch.from_numpy(moff.view(np.int64)).to(dev)
    d_grp = torch.from_numpy(grp.view(np.int32)).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    nb = int(moff[-1])
    d_rows = wire.group_rows(d_off, d_ids) if rows else None  # once per config
    t = time_region(lambda: wire.ingest(d_buf, nb, d_moff, d_grp, d_off, d_ids, rows=d_rows),
                    reps)
    # bytes read: message bytes + offset 8 + envelope group 4 + the group's
    # slot IDs 40 (5 x u64, read once per message); written: group 4, flags
    # 1, index/term/hint/log_term 32, status 1, type 1
    algo = nb + M * (8 + 4 + 40) + M * (4 + 1 + 32 + 1 + 1)
    if gpu_only:
        extra = {"unit": "messages/s", "bytes_per_message": nb / M}
        if reporter is not report:  # the default run's next_rows: the row's own parity
            ib, status, mtype = wire.ingest(d_buf, nb, d_moff, d_grp, d_off, d_ids, rows=d_rows)
            want = oc.ingest(buf, moff, grp, off, ids, threads=16)
            got = {"group": ib.group.cpu().numpy().view(np.uint32), "flags": ib.flags.cpu().numpy(),
                   "index": ib.index.cpu().numpy().view(np.uint64)[:M],
                   "term": ib.term.cpu().numpy().view(np.uint64)[:M],
                   "hint": ib.hint.cpu().numpy().view(np.uint64)[:M],
                   "log_term": ib.log_term.cpu().numpy().view(np.uint64)[:M],
                   "status": status.cpu().numpy()}
            bad = [n for n in got if not np.array_equal(got[n][:M], want[n])]
            extra["parity"] = "bit-exact" if not bad else "MISMATCH " + ", ".join(bad)
            extra["parity_check"] = (f"all {M} messages decoded by the device and by the C "
                                     "restatement of Message.Unmarshal + ingest "
                                     "(oracle/wire_oracle.c): every record column and status")
        reporter("wire ingest" + (" (group rows)" if rows else ""), M, t, algo, extra)
        return
    import time
    Ms = 1 << 22
    cpu = {}
    for threads in (16, 1):
        reps_c, t0 = 0, time.perf_counter()
        while True:
            oc.ingest(buf[: int(moff[Ms])], moff[: Ms + 1], grp[:Ms], off, ids, threads=threads)
            reps_c += 1
            if time.perf_counter() - t0 > 4:
                break
        cpu[threads] = reps_c * Ms / (time.perf_counter() - t0)
    reporter("wire ingest (raftpb.Message -> leader inbox)" + (", group rows" if rows else ""),
           M, t, algo,
           {"unit": "messages/s", "bytes_per_message": nb / M,
            "input_GBs": nb / t / 1e9,
            "cpu_baseline": {"value": cpu[16], "unit": "messages/s", "cores": 16, "kind": "port",
                             "value_1thread": cpu[1],
                             "sample": f"{Ms} messages of the same stream, C restatement of "
                                       "gogoproto Message.Unmarshal + ingest (oracle/wire_oracle.c)"}})


def _confchange_row_parity(table, op, cc_off, cc_type, cc_node, last, t, K):
    """The conf change row's expected result, checked whole on the device:
    every group's Simple(AddLearnerNode 6) over voters 1-5."""
    from etcd_amd.quorum.leader import PR_RECENT_ACTIVE
    nt, err, _ = table.change_soa(op, cc_off, cc_type, cc_node, last, fetch_errors=False)
    G = table.G
    S = 6 * G
    bad = []
    ar = torch.arange(S, device=dev)
    slot, g = ar % 6, ar // 6
    carried = slot < 5
    src = g * 5 + slot.clamp(max=4)
    checks = {
        "err": bool((err != 0).any()),
        "off": not torch.equal(nt.t["off"].long()[: G + 1],
                               torch.arange(0, S + 1, 6, device=dev)),
        "ids": not torch.equal(nt.t["ids"][:S], slot + 1),
        "cfg": not torch.equal(nt.t["cfg"][:G], t["cfg"]),
        "ext": not torch.equal(nt.t["ext"][:G], t["ext"]),
        "match": not torch.equal(nt.t["match"][:S], torch.where(carried, t["match"][src], 0)),
        "next": not torch.equal(nt.t["next"][:S], torch.where(carried, t["next"][src], last[g])),
        "pending_snapshot": not torch.equal(nt.t["pending_snapshot"][:S],
                                            torch.where(carried, t["pending_snapshot"][src], 0)),
        "pstate": not torch.equal(nt.t["pstate"][:S].long(),
                                  torch.where(carried, t["pstate"][src].long(),
                                              torch.full_like(ar, PR_RECENT_ACTIVE))),
        "infl_pos": not torch.equal(nt.t["infl_pos"][:S].long(),
                                    torch.where(carried, t["infl_pos"][src].long(), 0)),
        "infl_buf": not torch.equal(nt.t["infl_buf"][: S * K].view(S, K),
                                    torch.where(carried[:, None], t["infl_buf"].view(-1, K)[src], 0)),
    }
    bad = [k for k, v in checks.items() if v]
    del nt
    return "bit-exact" if not bad else "MISMATCH " + ", ".join(bad)


def confchange_config(G, reps, *, reporter=None, gpu_only=None):
    """§8f row 4: one Changer.Simple(AddLearnerNode) per group over G 5-voter
    groups (Progress carried for 5 slots, initialised for the new one),
    groups/s; CPU beside it: the Python restatement on a small sample."""
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    import time
    from etcd_amd.quorum.confchange import ConfigTable, ADD_LEARNER, SIMPLE
    from oracle import confchange_ref as CC
    K = 4
    S = 5 * G
    off = torch.arange(0, S + 1, 5, dtype=torch.int32, device=dev)
    ids = (torch.arange(S, dtype=torch.int64, device=dev) % 5) + 1
    t = {"off": off, "ids": ids,
         "cfg": torch.full((G,), 0x1F, dtype=torch.int32, device=dev),
         "ext": torch.zeros(G, dtype=torch.int32, device=dev),
         "match": torch.arange(S, dtype=torch.int64, device=dev),
         "next": torch.arange(S, dtype=torch.int64, device=dev) + 1,
         "pending_snapshot": torch.zeros(S, dtype=torch.int64, device=dev),
         "pstate": torch.full((S,), 1 | 8, dtype=torch.uint8, device=dev),
         "infl_pos": torch.zeros(S, dtype=torch.int32, device=dev),
         "infl_buf": torch.zeros(S * K, dtype=torch.int64, device=dev)}
    table = ConfigTable(G, S, K, t)
    op = torch.full((G,), SIMPLE, dtype=torch.uint8, device=dev)
    cc_off = torch.arange(G + 1, dtype=torch.int32, device=dev)
    cc_type = torch.full((G,), ADD_LEARNER, dtype=torch.uint8, device=dev)
    cc_node = torch.full((G,), 6, dtype=torch.int64, device=dev)
    last = torch.full((G,), 100, dtype=torch.int64, device=dev)
    tt = time_region(lambda: table.change_soa(op, cc_off, cc_type, cc_node, last,
                                              fetch_errors=False), reps)
    # read: off 4, ids 40, cfg/ext 8, op 1, cc_off 4, cc 9, last 8, Progress
    # 5 x (8+8+8+1+4+K*8); written: new_off 4, ids 48, cfg/ext 8, Progress
    # 6 x (29 + K*8), err 1, err_id 8
    pr = 29 + 8 * K
    algo = G * (4 + 40 + 8 + 1 + 4 + 9 + 8 + 5 * pr + 4 + 48 + 8 + 6 * pr + 9)
    if gpu_only:
        extra = {"unit": "groups/s"}
        if reporter is not report:  # the default run's next_rows: the row's own parity
            extra["parity"] = _confchange_row_parity(table, op, cc_off, cc_type, cc_node, last, t, K)
            extra["parity_check"] = (f"all {G} groups: Simple(AddLearnerNode 6) on voters 1-5 gives "
                                     "slots 1-6, the voter mask unchanged, slots 1-5's Progress "
                                     "and rings carried, slot 6 initProgress (confchange.go:"
                                     "258-281), no error — checked on the device")
        reporter("conf change", G, tt, algo, extra)
        return
    n = 20000
    trs = []
    for _ in range(n):
        tr = CC.Tracker.empty(K)
        tr.voters_in = {1, 2, 3, 4, 5}
        tr.prs = {i: CC.Pr(match=i, next=i + 1, state=1, recent_active=True) for i in range(1, 6)}
        trs.append(tr)
    t0 = time.perf_counter()
    for tr in trs:
        CC.Changer(tr, 100).simple([(CC.ADD_LEARNER, 6)])
    cpu1 = n / (time.perf_counter() - t0)
    reporter("conf change (Simple AddLearner, 5 -> 6 slots)", G, tt, algo,
           {"unit": "groups/s", "cpu_baseline": {
               "value": cpu1, "unit": "groups/s", "cores": 1, "kind": "port",
               "sample": f"{n} groups, Python restatement of confchange.Changer (oracle)"}})


def readindex_config(G, reps, Q=4, *, reporter=None, gpu_only=None):
    """§8f row 2: ReadIndex acks — two heartbeat responses per leader carrying
    the latest read context; the quorum releases all Q pending reads
    (MsgReadIndexResp / ReadState).  The read queues are restored before each
    step outside the timed launches (new MsgReadIndex requests are the
    host's).  Also CheckQuorum: QuorumActive over 16M CSR groups."""
    reporter = reporter or report
    gpu_only = GPU_ONLY if gpu_only is None else gpu_only
    from etcd_amd.quorum.leader import synth_readindex, readindex_inbox
    lg, last_ctx, pristine = synth_readindex(G, Q, device=dev)
    inboxes = [readindex_inbox(G, last_ctx, device=dev) for _ in range(reps + 2)]
    stats = torch.zeros(8, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream

    def timed(step):
        ev = HipEvents(2)
        times = []
        for k in range(reps + 2):
            for name, t0 in pristine.items():
                lg.t[name].copy_(t0)
            if k == 2:
                stats.zero_()
            ev.record(ev.ev[0], sp)
            step(inboxes[k])
            ev.record(ev.ev[1], sp)
            torch.cuda.synchronize()
            if k >= 2:
                times.append(ev.elapsed_ms(0, 1) / 1e3)
        ev.close()
        return float(np.median(times)), stats.cpu().tolist()
    t_ord, st = timed(lambda ib: lg.step(ib, msg_cap=8 * G, stats=stats, fetch=False))
    t_msg, st_ob = timed(lambda ib: lg.step_outbox(ib, stats=stats, fetch=False))
    assert st_ob[6] == st[6], "outbox and ordered forms generated different message counts"
    # the row's form: the outbox with its ReadState area — a local read's
    # answer is a ReadState (raft.go:1737-1745, Ready.ReadStates), not a message
    t, st_rs = timed(lambda ib: lg.step_outbox(ib, stats=stats, fetch=False, read_states=True))
    local_reads = (st[6] - st_rs[6]) / reps  # the ReadStates per step (out of the messages)
    # per group-step: 2 records 2 x 21 B, group state 84 B, 5 slots x 29 B,
    # read queue Q x 20 B read + written, the grouping scan 8 B; then the
    # answers: the row's form 40 B per message + 16 B per ReadState + two 4 B
    # counts per group; every answer a message (messages_*) 40 B each + a 4 B
    # count; the ordered form 40 B x 3 + the count scan 8 B per group
    base = G * (42 + 84 + 145 + Q * 20 * 2 + 8)
    algo = base + G * 8 + (st_rs[6] / reps) * 40 + local_reads * 16
    algo_msg = base + G * (4 + Q * 40)
    algo_ord = base + G * (8 + Q * 40 * 3)
    ordered = {"messages_us": t_msg * 1e6, "messages_algo_bytes": algo_msg,
               "messages_frac": algo_msg / t_msg / 1e9 / HBM_PEAK_GBS,
               "ordered_us": t_ord * 1e6, "ordered_algo_bytes": algo_ord,
               "ordered_frac": algo_ord / t_ord / 1e9 / HBM_PEAK_GBS,
               "read_states_per_step": local_reads,
               "form": "qb_dev_leader_step_outbox with its ReadState area (local answers as "
                       "16-byte ReadStates, follower answers as MsgReadIndexResp); messages_* = "
                       "the same outbox with every answer a message (rounds 4-5's row); "
                       "ordered_* = qb_dev_leader_step (group-ordered array)"}
    # CheckQuorum: QuorumActive over 16M groups (cfg u32 + active u16 -> u8)
    grp = batch.CsrGroups.synth(0x5EED0003, "ragged", 1 << 24, device=dev)
    active = torch.randint(-(1 << 15), 1 << 15, (1 << 24,), dtype=torch.int16, device=dev)
    tq = time_region(lambda: grp.quorum_active(active), 20)
    cq = {"read_queue": Q, "check_quorum_16M_us": tq * 1e6,
          "check_quorum_groups_per_s": (1 << 24) / tq,
          "check_quorum_GBs": (1 << 24) * 7 / tq / 1e9}
    if gpu_only:
        extra = {"unit": "group-steps/s", "reads_released_per_step": st[6] / reps, **cq, **ordered}
        if reporter is not report:  # the default run's next_rows: the row's own parity
            extra["parity"] = leader_row_parity("readindex")
            extra["parity_check"] = ("the same workload at 256K groups, ordered, outbox and "
                                     "outbox + ReadState forms vs the C oracle: queues, released "
                                     "reads, every message and ReadState")
        reporter("ReadIndex acks (leader step, heartbeat responses)", G, t, algo, extra)
        return
    # CPU beside it: the C restatement on 1M groups of the same workload
    import time
    from tests import oracle_c as oc
    Gs = 1 << 20
    lgc, ctxc, _ = synth_readindex(Gs, Q, device="cpu")
    ibc = readindex_inbox(Gs, ctxc, device="cpu")
    recc = {"group": ibc.group.numpy().view(np.uint32), "flags": ibc.flags.numpy(),
            "index": ibc.index.numpy().view(np.uint64), "term": ibc.term.numpy().view(np.uint64),
            "hint": ibc.hint.numpy().view(np.uint64),
            "log_term": ibc.log_term.numpy().view(np.uint64)}
    cpu = {}
    for threads in (16, 1):
        host = {k_: v.copy() for k_, v in lgc.numpy().items()}
        t1 = time.perf_counter()
        oc.leader_step(host, lgc.inflight_cap, Q, 0, recc, threads=threads, msg_cap=8 * Gs)
        cpu[threads] = Gs / (time.perf_counter() - t1)
    reporter("ReadIndex acks (leader step, heartbeat responses)", G, t, algo,
           {"unit": "group-steps/s", "reads_released_per_step": st[6] / reps, **ordered,
            "cpu_baseline": {"value": cpu[16], "unit": "group-steps/s", "cores": 16,
                             "kind": "port", "value_1thread": cpu[1],
                             "sample": f"{Gs} groups, one step, C restatement (oracle)"},
            **cq})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="3,4,5")
    ap.add_argument("--gpu-only", action="store_true",
                    help="leader, wire, confchange: skip the CPU baseline (A/B)")
    ap.add_argument("--lab-lib", default=None,
                    help="A/B runs: bind this libquorumbatch.so build (etcd_amd._lib.use_lab_library)")
    a = ap.parse_args()
    if a.lab_lib:
        from etcd_amd import _lib
        _lib.use_lab_library(a.lab_lib)
    global GPU_ONLY
    GPU_ONLY = a.gpu_only
    which = set(a.only.split(","))
    if "1" in which:
        plumbing_config(a.reps)
    if "3" in which:
        csr_config("ragged", 1 << 24, a.reps)
    if "4" in which:
        csr_config("joint", 1 << 23, a.reps)
    if "5" in which:
        tracker_config(1 << 24, a.reps)
    if "leader" in which:
        leader_config(1 << 22, a.reps)
    if "leader-sorted" in which:  # development: records already in group order
        leader_config(1 << 22, a.reps, shuffle=False)
    if "wire" in which:  # with the group-row table (the configuration-time cache)
        wire_config(1 << 24, a.reps, rows=True)
    if "wire-csr" in which:  # gathering off + ids per message
        wire_config(1 << 24, a.reps)
    if "wire-g4k" in which:  # development: 4096 groups (group rows cache-resident)
        wire_config(1 << 24, a.reps, G=4096)
    if "readindex" in which:
        readindex_config(1 << 22, a.reps)
    if "confchange" in which:
        confchange_config(1 << 23, a.reps)
    if "wire-tracker" in which:
        wire_tracker_config(1 << 24, a.reps)
    if "wire-tracker-fused" in which:  # development A/B: the one call alone
        wire_tracker_config(1 << 24, a.reps, fused_only=True)
    if "wire-tracker-csr" in which:  # the composed tick over configs[2]'s ragged CSR groups
        wire_tracker_config(1 << 24, a.reps, csr=True)


if __name__ == "__main__":
    main()
