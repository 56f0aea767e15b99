"""The composed per-tick path in one call (qb_dev_ingest_fixed_tracker_step,
etcd_amd/csrc/qb_wire_tracker.hip) against the chain of C oracles: the
restated Message.Unmarshal (oracle/wire_oracle.c, raft.pb.go:1739-2061) and
the sequential stepLeader MsgAppResp case (oracle/quorum_oracle.c,
raft.go:847-921, 1100-1109, 1237-1259; progress.go:144-153; log.go:328-334)
on the decoded records, with the fused entry's contract applied to them: a
message that is not a decoded MsgAppResp steps nothing (counted as a bad
group) and a From without Progress counts as a non-member."""
import os
import random
import sys

import numpy as np
import pytest

from oracle import raftpb_ref as W
from tests import oracle_c as oc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _chain_oracle(n, G, buf, moff, grp, off, ids, st):
    """C decode, the fused contract on its records, the sequential tracker."""
    want = oc.ingest(buf, moff, grp, off, ids, threads=8, nbytes=buf.size)
    g = want["group"].copy()
    f = want["flags"].copy()
    notrec = (want["status"] != 0) | (((f >> 4) & 3) != 0)
    g[notrec] = 0xFFFFFFFF
    nonm = ~notrec & ((f & 0x40) != 0)
    f[nonm] = (f[nonm] & 0xF0) | 0x0F  # slot 15 >= n: a non-member
    stats = oc.appresp_sequential(n, G, (g, f, want["index"], want["term"]), st, threads=8)
    return want["status"], stats


def _host_state(tr, G):
    return {"match": _u64(tr.match).copy(),
            "active": tr.active.cpu().numpy().view(np.uint16)[:G].copy(),
            "term": _u64(tr.term).copy(), "term_start": _u64(tr.term_start).copy(),
            "committed": _u64(tr.committed).copy(), "stepped_down": np.zeros(G, np.uint8)}


def _check(tr, G, st, stats_dev, stats_want):
    assert np.array_equal(_u64(tr.match), st["match"])
    assert np.array_equal(_u64(tr.committed), st["committed"])
    assert np.array_equal(tr.active.cpu().numpy().view(np.uint16)[:G], st["active"])
    sd = tr.stepdown_at.cpu().numpy().view(np.uint32)
    assert np.array_equal(sd != 0xFFFFFFFF, st["stepped_down"] != 0)
    assert np.array_equal(stats_dev[:7], stats_want[:7].astype(np.int64)), (stats_dev, stats_want)


def test_fused_tick_vs_chain_of_c_oracles():
    """The bench row's workload (tools/bench_configs.py wire_tracker_tick:
    canonical MsgAppResp, leader terms 20006-20007: side records) at 64K
    groups over three ticks, against the C chain; and the same ticks through
    the device chain (ingest + tracker step) reach the same state."""
    import torch
    from etcd_amd.quorum import batch, wire
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs as bc
    G, n = 1 << 16, 5
    tr, snap, ticks, rows, off, ids = bc.wire_tracker_tick(G, 3, dev_=torch.device("cuda"))
    st = _host_state(tr, G)
    h_off, h_ids = off.cpu().numpy().view(np.uint32), _u64(ids)
    wst = torch.zeros(4, dtype=torch.int64, device="cuda")
    for buf, nbytes, moff, grp, _direct in ticks:
        status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows, wire_stats=wst)
        want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], _u64(moff),
                                                grp.cpu().numpy().view(np.uint32), h_off, h_ids, st)
        assert np.array_equal(status.cpu().numpy(), want_status)
        _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)
    assert int(wst[0].item()) == 3 * G and int(wst[1:].sum().item()) == 0
    fused = {k: getattr(tr, k).clone() for k in snap}
    for k, v in snap.items():
        getattr(tr, k).copy_(v)
    for buf, nbytes, moff, grp, _direct in ticks:
        ib, status, _ = wire.ingest(buf, nbytes, moff, grp, off, ids, rows=rows)
        tr.step(batch.AppRespBatch(ib.group, ib.flags, ib.index, ib.term))
    for k in snap:
        assert torch.equal(getattr(tr, k), fused[k]), k
    assert int((st["committed"] > 0).sum()) > G // 2


def _mixed_tick(r, G, n, gterm, ids_of, k, hot=None, big_waves=0):
    """One tick of M = 4G messages of every kind the fused path must tell
    apart, host-encoded (oracle/raftpb_ref.py marshal_message)."""
    M = 4 * G
    msgs, grps = [], []
    for i in range(M):
        g = hot if hot is not None and r.random() < 0.3 else r.randrange(G)
        ids = ids_of(g)
        s = r.randrange(n)
        t = int(gterm[g])
        x = r.random()
        term = t - 1 if x < 0.04 and t > 0 else t + 1 if x < 0.045 else t
        idx = (1 << 30) + g * 97 + k * 64 + r.randrange(200)
        if r.random() < 0.02:
            idx = (1 << 41) + g  # past the record's 40-bit index: an escape
        rej = r.random() < 0.1
        y = r.random()
        if y < 0.05:     # heartbeat response: decoded, not stepped
            b = W.marshal_message(9, ids[0], ids[s], term, 0, 0, (), 0, W.EMPTY_SNAPSHOT, False, 0,
                                  r.getrandbits(63).to_bytes(8, "big") if r.random() < 0.5 else None)
        elif y < 0.10:   # From without Progress
            b = W.marshal_message(4, ids[0], 999_999_999 + i, term, 0, idx, (), 0, W.EMPTY_SNAPSHOT,
                                  rej, 0, None)
        elif y < 0.14:   # non-canonical (a field moved to the front): the generic decoder
            b = W._key(6, 0) + W.varint(idx) + W.marshal_message(4, ids[0], ids[s], term, 0, idx,
                                                                (), 0, W.EMPTY_SNAPSHOT, rej, 0)
        elif y < 0.16:   # truncated: an unmarshal error
            full = W.marshal_message(4, ids[0], ids[s], term, 0, idx, (), 0, W.EMPTY_SNAPSHOT, rej, 0)
            b = full[: r.randrange(1, len(full))]
        elif y < 0.17:   # another message type
            b = W.marshal_message(3, ids[0], ids[s], term, 0, idx)
        else:
            b = W.marshal_message(4, ids[0], ids[s], term, 0, idx, (), 0, W.EMPTY_SNAPSHOT, rej, 0)
        if r.random() < 0.01:
            g = G + r.randrange(5)  # envelope group past the shard
        msgs.append(b)
        grps.append(g)
    # whole waves of large messages (entries): past a wave's LDS slice
    for w in range(big_waves):
        base = r.randrange(M // 64) * 64
        for j in range(64):
            g = grps[base + j] % G
            ids = ids_of(g)
            ent = W.marshal_entry(1, 2, 0, bytes(120))
            msgs[base + j] = W.marshal_message(4, ids[0], ids[1 + j % (n - 1)], int(gterm[g]), 0,
                                               (1 << 30) + g * 97 + k * 64 + 300, (ent,))
            grps[base + j] = g
    return msgs, grps


@pytest.mark.parametrize("large_frac,hot,big_waves", [(0.05, False, 0), (0.6, False, 3),
                                                      (0.6, True, 0), (0.0, False, 2)])
def test_fused_mixed_stream_vs_chain_of_c_oracles(large_frac, hot, big_waves):
    """Every kind of message in one stream — stale / higher-term (the slow
    path re-decodes its chunk) / rejects, heartbeat responses and another
    type, non-members, groups past the shard, non-canonical encodings and
    whole waves of large messages (the deferred launch), truncations,
    indexes past 2^40 and terms past 2^32 (escapes) — with group terms small,
    past the record's term field (side records when dense in a tile, escapes
    when rare: large_frac) and past 2^32; hot: 30 % of a tick on one group
    (K4 folds it).  Four ticks against the C chain, state and every stat."""
    import torch
    from etcd_amd.quorum import batch, wire
    r = random.Random(int(large_frac * 100) + 7 * hot + big_waves)
    G, n = 1 << 12, 5
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (1000 + np.arange(n * G, dtype=np.uint64) * 3)  # ascending per group
    ids_of = lambda g: [int(v) for v in ids[n * g: n * g + n]]  # noqa: E731
    gterm = np.where(np.array([r.random() < large_frac for _ in range(G)]),
                     np.array([r.randrange(2048, 1 << 20) for _ in range(G)], np.uint64),
                     np.uint64(7)).astype(np.uint64)
    gterm[: G // 64] = (1 << 33) + np.arange(G // 64, dtype=np.uint64)  # past 2^32: escapes
    dev = torch.device("cuda")
    tr = batch.FixedTracker(n, G, dev)
    tr.term.copy_(torch.from_numpy(gterm.view(np.int64)))
    tr.term_start.fill_(1 << 30)
    tr.match[0].fill_((1 << 31))
    for s in range(1, n):
        tr.match[s].copy_(torch.from_numpy(((1 << 30) + np.arange(G, dtype=np.int64) * 97)))
    tr.commit_advance()
    st = _host_state(tr, G)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    rows = wire.group_rows(d_off, d_ids)
    wst = torch.zeros(4, dtype=torch.int64, device=dev)
    want_w = np.zeros(4, np.int64)
    for k in range(4):
        msgs, grps = _mixed_tick(r, G, n, gterm, ids_of, k, hot=r.randrange(G) if hot else None,
                                 big_waves=big_waves)
        buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
        status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows, wire_stats=wst)
        want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], _u64(moff),
                                                grp.cpu().numpy().view(np.uint32), off, ids, st)
        assert np.array_equal(status.cpu().numpy(), want_status)
        want_w += np.bincount(want_status, minlength=4)[:4]
        _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)
        # the higher-term records stepped some groups down: re-arm them
        tr.stepdown_at.fill_(-1)
        st["stepped_down"][:] = 0
    assert np.array_equal(wst.cpu().numpy(), want_w)


@pytest.mark.parametrize("n", [9, 16, 1])
def test_fused_off_ids_and_empty(n):
    """off + ids instead of the row table (a member past the row's 7 read from
    ids), and M = 0 (the tracker still runs maybeCommit, as the step); the
    widest fixed config and a single voter."""
    import torch
    from etcd_amd.quorum import batch, wire
    r = random.Random(5 + n)
    G = 1 << 10
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (50 + np.arange(n * G, dtype=np.uint64) * 2)
    dev = torch.device("cuda")
    tr = batch.FixedTracker(n, G, dev)
    tr.term.fill_(3)
    tr.term_start.fill_(10)
    st = _host_state(tr, G)
    msgs, grps = [], []
    for i in range(3 * G):
        g = r.randrange(G)
        s = r.randrange(n)
        msgs.append(W.marshal_message(4, int(ids[n * g]), int(ids[n * g + s]), 3, 0,
                                      20 + r.randrange(100), (), 0, W.EMPTY_SNAPSHOT,
                                      r.random() < 0.1, 0))
        grps.append(g)
    buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, off=d_off, ids=d_ids)
    want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], _u64(moff),
                                            grp.cpu().numpy().view(np.uint32), off, ids, st)
    assert np.array_equal(status.cpu().numpy(), want_status)
    _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)
    if n > 8:
        assert int((st["match"][8] > 0).sum()) > 0  # slot 8: past the 7 IDs a row holds
    empty = torch.zeros(1, dtype=torch.uint8, device=dev)
    mo = torch.zeros(1, dtype=torch.int64, device=dev)
    eg = torch.zeros(0, dtype=torch.int32, device=dev)
    wire.ingest_tracker_step(tr, empty, 0, mo, eg, off=d_off, ids=d_ids)
    assert np.array_equal(_u64(tr.committed), st["committed"])


@pytest.mark.parametrize("kind,term_base", [("ragged", 0), ("joint", 20000), ("ragged", 1 << 33)])
def test_fused_csr_vs_chain_of_c_oracles(kind, term_base):
    """qb_dev_ingest_csr_tracker_step: ragged voters + learners and joint
    configs (oracle/quorum_oracle.c gen_csr), the groups' slot IDs over the
    tracker's own off, stale / higher-term / rejected responses, non-members,
    envelope groups past the shard, heartbeat responses and non-canonical
    encodings, group terms small, past the record's field and past 2^32 —
    three ticks against the C chain (restated Unmarshal, then the sequential
    CSR tracker oracle), state and every stat."""
    import torch
    from etcd_amd.quorum import batch, wire
    from tests.test_gpu_tracker_csr import _batch, _state, _tracker
    G, M = 3000, 12000
    rng = np.random.default_rng(G + term_base % 997)
    r = random.Random(term_base % 991)
    off, cfg, sizes, st = _state(rng, kind, G, term_base)
    tr = _tracker(off, cfg, st, track_next=False)
    st.pop("next")
    ids = (100 + 3 * np.arange(int(off[-1]), dtype=np.uint64)).astype(np.uint64)
    d_ids = torch.from_numpy(ids.view(np.int64)).to("cuda")
    wst = torch.zeros(4, dtype=torch.int64, device="cuda")
    want_w = np.zeros(4, np.int64)
    for tick in range(3):
        group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, st, stale=0.05,
                                                      higher=0.003, reject=0.1, nonmember=0.02,
                                                      bad=0.01)
        msgs, grps = [], []
        for i in range(M):
            g = int(group[i])
            gi = g if g < G else 0
            s0, n_g = int(off[gi]), int(sizes[gi])
            frm = int(ids[s0 + int(slot[i])]) if int(slot[i]) < n_g else 999_999_999 + i
            to = int(ids[s0]) if n_g else 1
            y = r.random()
            if y < 0.04:
                b = W.marshal_message(9, to, frm, int(term[i]), 0, 0, (), 0, W.EMPTY_SNAPSHOT,
                                      False, 0, None)
            elif y < 0.08:
                b = W._key(6, 0) + W.varint(int(index[i])) + W.marshal_message(
                    4, to, frm, int(term[i]), 0, int(index[i]), (), 0, W.EMPTY_SNAPSHOT,
                    bool(rej[i]), 0)
            else:
                b = W.marshal_message(4, to, frm, int(term[i]), 0, int(index[i]), (), 0,
                                      W.EMPTY_SNAPSHOT, bool(rej[i]), 0)
            msgs.append(b)
            grps.append(g)
        buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device="cuda")
        status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, ids=d_ids, wire_stats=wst)
        want = oc.ingest(buf.cpu().numpy()[:nbytes], _u64(moff), grp.cpu().numpy().view(np.uint32),
                         off, ids, threads=8)
        assert np.array_equal(status.cpu().numpy(), want["status"])
        want_w += np.bincount(want["status"], minlength=4)[:4]
        g2 = want["group"].copy()
        f2 = want["flags"].copy()
        notrec = (want["status"] != 0) | (((f2 >> 4) & 3) != 0)
        g2[notrec] = 0xFFFFFFFF
        nonm = ~notrec & ((f2 & 0x40) != 0)
        f2[nonm] = (f2[nonm] & 0xF0) | 0x0F
        stats = oc.csr_appresp_sequential(off, cfg, (g2, f2, want["index"], want["term"]), st)
        S = st["match"].size
        assert np.array_equal(batch.as_u64(tr.match)[:S], st["match"]), tick
        assert np.array_equal(tr.active.cpu().numpy().view(np.uint16)[:G], st["active"]), tick
        assert np.array_equal(batch.as_u64(tr.committed), st["committed"]), tick
        assert np.array_equal(tr.stepped_down().cpu().numpy(), st["stepped_down"].astype(bool))
        assert tr.stats.cpu().numpy()[:7].tolist() == [int(x) for x in stats[:7]], tick
        tr.stepdown_at.fill_(-1)
        st["stepped_down"][:] = 0
    assert np.array_equal(wst.cpu().numpy(), want_w)


def test_fused_unaligned_buffer_and_input_checks():
    """The message bytes at an address that is not 16-byte aligned (a view
    into a larger buffer: the decoder stages its byte slices with plain loads
    instead of LDS-DMA) give the same status and state as the aligned copy;
    short or mistyped inputs raise before any device call."""
    import torch
    from etcd_amd import _lib
    from etcd_amd.quorum import batch, wire
    r = random.Random(11)
    G, n = 1 << 11, 5
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (7 + np.arange(n * G, dtype=np.uint64) * 5)
    dev = torch.device("cuda")
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    rows = wire.group_rows(d_off, d_ids)
    msgs, grps = [], []
    for _ in range(5 * G + 37):  # a partial last tile
        g = r.randrange(G)
        s = r.randrange(n)
        msgs.append(W.marshal_message(4, int(ids[n * g]), int(ids[n * g + s]), 9, 0,
                                      100 + r.randrange(1000), (), 0, W.EMPTY_SNAPSHOT,
                                      r.random() < 0.1, 0))
        grps.append(g)
    buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
    outs = []
    for shift in (0, 3, 8):
        tr = batch.FixedTracker(n, G, dev)
        tr.term.fill_(9)
        tr.term_start.fill_(50)
        b = buf
        if shift:
            host = torch.zeros(nbytes + 32, dtype=torch.uint8, device=dev)
            b = host[shift:shift + nbytes]
            b.copy_(buf[:nbytes])
            assert b.data_ptr() % 16 != 0
        wst = torch.zeros(4, dtype=torch.int64, device=dev)
        status = wire.ingest_tracker_step(tr, b, nbytes, moff, grp, rows=rows, wire_stats=wst)
        outs.append((status.cpu(), batch.as_u64(tr.match).copy(), batch.as_u64(tr.committed).copy(),
                     tr.stats.cpu().clone(), wst.cpu()))
        if shift == 0:
            st = _host_state(tr, G)
            st["match"][:] = 0
            st["committed"][:] = 0
            st["active"][:] = 0
            want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], _u64(moff),
                                                    grp.cpu().numpy().view(np.uint32), off, ids, st)
            assert np.array_equal(status.cpu().numpy(), want_status)
            _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0])
        assert np.array_equal(o[1], outs[0][1]) and np.array_equal(o[2], outs[0][2])
        assert torch.equal(o[3], outs[0][3]) and torch.equal(o[4], outs[0][4])
    tr = batch.FixedTracker(n, G, dev)
    bad = [lambda: wire.ingest_tracker_step(tr, buf[: nbytes - 1], nbytes, moff, grp, rows=rows),
           lambda: wire.ingest_tracker_step(tr, buf.view(torch.int8), nbytes, moff, grp, rows=rows),
           lambda: wire.ingest_tracker_step(tr, buf, nbytes, moff[:-1], grp, rows=rows),
           lambda: wire.ingest_tracker_step(tr, buf, nbytes, moff, grp.to(torch.int64), rows=rows),
           lambda: wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows[:-8]),
           lambda: wire.ingest_tracker_step(tr, buf, -1, moff, grp, rows=rows),
           lambda: wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows,
                                            wire_stats=torch.zeros(3, dtype=torch.int64, device=dev)),
           lambda: wire.ingest(buf[:10], nbytes, moff, grp, d_off, d_ids),
           lambda: wire.ingest(buf, nbytes, moff, grp, d_off.to(torch.int64), d_ids),
           lambda: wire.ingest(buf, nbytes, moff, grp, d_off, d_ids, rows=rows[:8])]
    for i, call in enumerate(bad):
        with pytest.raises(_lib.QuorumBatchError):
            call()


def test_corrupt_offsets_ingest_and_fused():
    """msg_off from a broken caller: an end before its start, a last offset
    past the buffer and an aligned block of 257 offsets far past it (whole
    waves and ingest workgroups whose staged span starts beyond the buffer:
    nothing may be staged from there).  Both the ingest and the composed call
    report what the restated Unmarshal does (UNMARSHAL for a slice outside
    the buffer), and the tracker steps what is left."""
    import torch
    from etcd_amd.quorum import batch, wire
    r = random.Random(21)
    G, n = 1 << 11, 5
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (11 + np.arange(n * G, dtype=np.uint64) * 7)
    dev = torch.device("cuda")
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    rows = wire.group_rows(d_off, d_ids)
    msgs, grps = [], []
    for _ in range(4 * G):
        g = r.randrange(G)
        s = r.randrange(n)
        msgs.append(W.marshal_message(4, int(ids[n * g]), int(ids[n * g + s]), 4, 0,
                                      30 + r.randrange(500), (), 0, W.EMPTY_SNAPSHOT,
                                      r.random() < 0.1, 0))
        grps.append(g)
    buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
    h = _u64(moff).copy()
    M = len(msgs)
    for i in (5, 900, 3001):  # message i - 1 spans two messages, message i ends before it starts
        h[i], h[i + 1] = h[i + 1], h[i]
    h[M] = nbytes + 1000  # the last message ends past the buffer
    h[1024:1024 + 257] = nbytes + (1 << 20) + np.arange(257, dtype=np.uint64) * 40
    moff = torch.from_numpy(h.view(np.int64)).to(dev)
    ib, status, _ = wire.ingest(buf, nbytes, moff, grp, d_off, d_ids, rows=rows)
    want = oc.ingest(buf.cpu().numpy()[:nbytes], h, grp.cpu().numpy().view(np.uint32), off, ids,
                     threads=8, nbytes=nbytes)
    got = status.cpu().numpy()
    assert np.array_equal(got, want["status"])
    assert (got[1024:1024 + 257] == wire.WIRE_UNMARSHAL).all() and got[M - 1] == wire.WIRE_UNMARSHAL
    assert np.array_equal(ib.group.cpu().numpy().view(np.uint32)[:M], want["group"])
    tr = batch.FixedTracker(n, G, dev)
    tr.term.fill_(4)
    tr.term_start.fill_(20)
    st = _host_state(tr, G)
    status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows)
    want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], h,
                                            grp.cpu().numpy().view(np.uint32), off, ids, st)
    assert np.array_equal(status.cpu().numpy(), want_status)
    _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)


@pytest.mark.parametrize("all_empty", [True, False])
def test_empty_messages_ingest_and_fused(all_empty):
    """Zero-length messages (an empty slice unmarshals to a default Message:
    type MsgHup, not a response) — every message empty with no bytes at all,
    or one in three empty between real responses — through the ingest and
    the composed call, against the C oracle."""
    import torch
    from etcd_amd.quorum import batch, wire
    r = random.Random(31 + all_empty)
    G, n = 1 << 10, 5
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (3 + np.arange(n * G, dtype=np.uint64) * 2)
    dev = torch.device("cuda")
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    rows = wire.group_rows(d_off, d_ids)
    msgs, grps = [], []
    for i in range(3 * G + 5):
        g = r.randrange(G)
        if all_empty or i % 3 == 0:
            msgs.append(b"")
        else:
            msgs.append(W.marshal_message(4, int(ids[n * g]), int(ids[n * g + r.randrange(n)]), 2,
                                          0, 10 + r.randrange(100), (), 0, W.EMPTY_SNAPSHOT,
                                          False, 0))
        grps.append(g)
    buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
    h_moff, h_grp = _u64(moff), grp.cpu().numpy().view(np.uint32)
    want = oc.ingest(buf.cpu().numpy()[:nbytes], h_moff, h_grp, off, ids, threads=8, nbytes=nbytes)
    _, status, _ = wire.ingest(buf, nbytes, moff, grp, d_off, d_ids, rows=rows)
    assert np.array_equal(status.cpu().numpy(), want["status"])
    assert (want["status"][[i for i, m in enumerate(msgs) if not m]] == wire.WIRE_TYPE).all()
    tr = batch.FixedTracker(n, G, dev)
    tr.term.fill_(2)
    tr.term_start.fill_(5)
    st = _host_state(tr, G)
    status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows)
    want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], h_moff, h_grp, off,
                                            ids, st)
    assert np.array_equal(status.cpu().numpy(), want_status)
    _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)


@pytest.mark.parametrize("G", [1, 64])
def test_fused_few_groups_many_records(G):
    """A tick of 2^16 responses over one group or 64: one super-bucket takes
    every record (its regions run past their reserved cap into the pool when
    they fill) and K4 folds a thousand or more records per group — the
    composed call against the C chain."""
    import torch
    from etcd_amd.quorum import batch, wire
    r = random.Random(41 + G)
    n = 5
    off = np.arange(0, n * G + 1, n, dtype=np.uint32)
    ids = (9 + np.arange(n * G, dtype=np.uint64) * 4)
    dev = torch.device("cuda")
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    rows = wire.group_rows(d_off, d_ids)
    msgs, grps = [], []
    for _ in range(1 << 16):
        g = r.randrange(G)
        msgs.append(W.marshal_message(4, int(ids[n * g]), int(ids[n * g + r.randrange(n)]),
                                      6 if r.random() < 0.98 else 5, 0, 100 + r.randrange(5000), (),
                                      0, W.EMPTY_SNAPSHOT, r.random() < 0.05, 0))
        grps.append(g)
    buf, nbytes, moff, grp = wire.pack_messages(msgs, grps, device=dev)
    tr = batch.FixedTracker(n, G, dev)
    tr.term.fill_(6)
    tr.term_start.fill_(50)
    st = _host_state(tr, G)
    wst = torch.zeros(4, dtype=torch.int64, device=dev)
    status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows, wire_stats=wst)
    want_status, want_stats = _chain_oracle(n, G, buf.cpu().numpy()[:nbytes], _u64(moff),
                                            grp.cpu().numpy().view(np.uint32), off, ids, st)
    assert np.array_equal(status.cpu().numpy(), want_status)
    _check(tr, G, st, tr.stats.cpu().numpy(), want_stats)
    assert int(wst[0].item()) == len(msgs)
