"""GPU parity of wire ingest (qb_dev_ingest_messages) against the raftpb
restatement (oracle/raftpb_ref.py, itself checked against Google's protobuf
runtime): valid messages of every field shape, malformed and mutated bytes
(every Unmarshal error path), non-members, contexts; then decode + leader
step end to end against the leader oracle."""
import copy
import random

import numpy as np
import pytest

from oracle import leader_ref as L
from oracle import raftpb_ref as W
from tests import leader_pack as LP
from tests.wire_gen import groups_ids as _groups_ids, random_message as _random_message

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,rows", [(1, False), (2, False), (1, True), (3, True)])
def test_ingest_matches_oracle(seed, rows):
    import torch
    from etcd_amd.quorum import wire
    r = random.Random(seed)
    G = 500
    off, ids = _groups_ids(r, G)
    msgs, groups = [], []
    for _ in range(20000):
        g = r.randrange(G + 3)  # a few envelope groups past G
        gids = ids[off[g]:off[g + 1]].tolist() if g < G else []
        msgs.append(_random_message(r, gids))
        groups.append(g)
    buf, nb, moff, mg = wire.pack_messages(msgs, groups)
    stats = torch.zeros(4, dtype=torch.int64, device="cuda")
    d_off = torch.from_numpy(off.view(np.int32)).cuda()
    d_ids = torch.from_numpy(ids.view(np.int64)).cuda()
    ib, status, mtype = wire.ingest(buf, nb, moff, mg, d_off, d_ids, stats,
                                    rows=wire.group_rows(d_off, d_ids) if rows else None)
    got = list(zip(status.cpu().numpy().tolist(), ib.group.cpu().numpy().view(np.uint32).tolist(),
                   ib.flags.cpu().numpy().tolist(),
                   ib.index.cpu().numpy().view(np.uint64).tolist(),
                   ib.term.cpu().numpy().view(np.uint64).tolist(),
                   ib.hint.cpu().numpy().view(np.uint64).tolist(),
                   ib.log_term.cpu().numpy().view(np.uint64).tolist()))
    types = mtype.cpu().numpy().tolist()
    counts = [0, 0, 0, 0]
    for i, (b, g) in enumerate(zip(msgs, groups)):
        gids = ids[off[g]:off[g + 1]].tolist() if g < G else []
        want = W.ingest(b, g, gids)
        counts[want[0]] += 1
        assert got[i] == tuple(want[:7]), (i, b.hex(), got[i], want)
        if want[0] != W.ST_UNMARSHAL:
            assert types[i] == want[7] & 0xFF, i
    assert stats.cpu().tolist() == counts
    assert min(counts) > 0  # every status exercised


def test_ingest_then_leader_step_end_to_end():
    """Encode a random leader batch as raftpb bytes, ingest on the device, run
    the leader step on the decoded records: identical to the oracle on the
    original records."""
    import torch
    from etcd_amd.quorum import wire
    from etcd_amd.quorum.leader import LeaderGroups
    rng = np.random.default_rng(5)
    groups = LP.random_groups(rng, 400, 4, 3, max_slots=9)
    recs = LP.random_records(rng, groups, 1500, bad_frac=0)
    node_ids = [sorted(rng.choice(np.arange(1, 1000), g.n_slots, replace=False).tolist())
                for g in groups]
    msgs, env = [], []
    for gi, m in recs:
        frm = node_ids[gi][m.slot] if m.slot < groups[gi].n_slots else 5000
        t = {0: 4, 1: 9, 2: 11, 3: 10}[m.kind]
        ctx = None
        if m.kind == 1 and m.index:
            ctx = m.index.to_bytes(8, "big")
        idx = 0 if m.kind == 1 else m.index
        msgs.append(W.marshal_message(t, 1, frm, m.term, m.log_term, idx, reject=m.reject,
                                      reject_hint=m.hint, context=ctx))
        env.append(gi)
    off = np.zeros(len(groups) + 1, np.uint32)
    off[1:] = np.cumsum([g.n_slots for g in groups])
    ids = np.array([x for l in node_ids for x in l], np.uint64)
    buf, nb, moff, mg = wire.pack_messages(msgs, env)
    ib, status, _ = wire.ingest(buf, nb, moff, mg, torch.from_numpy(off.view(np.int32)).cuda(),
                                torch.from_numpy(ids.view(np.int64)).cuda())
    assert int(status.max().item()) == 0
    eng = LeaderGroups(LP.pack(groups, 4, 3), 4, 3, 0, device="cuda")
    res = eng.step(ib)
    orc = copy.deepcopy(groups)
    for g in orc:
        g.msgs = []
    L.run_batch(orc, recs)
    dev = copy.deepcopy(groups)
    LP.unpack_into(dev, eng.numpy(), 4, 3)
    assert [LP.state_key(g) for g in dev] == [LP.state_key(g) for g in orc]
    want = [(gi,) + m.key() for gi, g in enumerate(orc) for m in g.msgs]
    got = [(int(m["group"]), int(m["type"]), int(m["to"]), int(m["index"]), int(m["log_term"]),
            int(m["commit"]), int(m["aux"])) for m in res.msgs]
    assert got == want


@pytest.mark.parametrize("rows", [False, True])
def test_response_stream_full_size_vs_c_oracle(rows):
    """The bench workload (4M gogoproto-encoded responses to 1M leaders)
    decoded on the device (CSR slot IDs, or the 64-byte group rows) and by the
    C restatement: every column identical."""
    import torch
    from etcd_amd.quorum import wire
    from tests import oracle_c as oc
    M, G = 1 << 22, 1 << 20
    buf, moff, grp, off, ids = wire.synth_response_stream(M, G)
    dev = "cuda"
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    ib, status, _ = wire.ingest(torch.from_numpy(buf).to(dev), int(moff[-1]),
                                torch.from_numpy(moff.view(np.int64)).to(dev),
                                torch.from_numpy(grp.view(np.int32)).to(dev), d_off, d_ids,
                                rows=wire.group_rows(d_off, d_ids) if rows else None)
    want = oc.ingest(buf, moff, grp, off, ids, threads=16)
    assert np.array_equal(status.cpu().numpy(), want["status"])
    assert int(want["status"].max()) == 0
    assert np.array_equal(ib.group.cpu().numpy().view(np.uint32), want["group"])
    assert np.array_equal(ib.flags.cpu().numpy(), want["flags"])
    for col in ("index", "term", "hint", "log_term"):
        assert np.array_equal(getattr(ib, col).cpu().numpy().view(np.uint64), want[col]), col


def test_ingest_then_tracker_step_vs_c_oracles():
    """The composed per-tick chain (bench next_rows "wire -> tracker tick"):
    device-encoded MsgAppResp bytes, decoded by the device and by the C
    restatement of Message.Unmarshal (oracle/wire_oracle.c); the device's
    records through qb_dev_fixed_tracker_step over three ticks, against the
    sequential C oracle of stepLeader's MsgAppResp case on the C decoder's
    records: match, committed, active, stepped-down identical."""
    import os
    import sys
    import torch
    from etcd_amd.quorum import batch, wire
    from tests import oracle_c as oc
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import bench_configs as bc
    G, n = 1 << 16, 5
    tr, snap, ticks, rows, off, ids = bc.wire_tracker_tick(G, 3, dev_=torch.device("cuda"))
    u64 = lambda t: t.cpu().numpy().view(np.uint64)
    st = {"match": u64(tr.match).copy(), "active": tr.active.cpu().numpy().view(np.uint16)[:G].copy(),
          "term": u64(tr.term).copy(), "term_start": u64(tr.term_start).copy(),
          "committed": u64(tr.committed).copy(), "stepped_down": np.zeros(G, np.uint8)}
    h_off = off.cpu().numpy().view(np.uint32)
    h_ids = u64(ids)
    for buf, nbytes, moff, grp, _direct in ticks:
        ib, status, _ = wire.ingest(buf, nbytes, moff, grp, off, ids, rows=rows)
        assert int(status.max().item()) == 0
        want = oc.ingest(buf.cpu().numpy(), u64(moff), grp.cpu().numpy().view(np.uint32),
                         h_off, h_ids, threads=8)
        assert np.array_equal(ib.group.cpu().numpy().view(np.uint32), want["group"])
        assert np.array_equal(ib.flags.cpu().numpy(), want["flags"])
        assert np.array_equal(u64(ib.index), want["index"])
        assert np.array_equal(u64(ib.term), want["term"])
        tr.step(batch.AppRespBatch(ib.group, ib.flags, ib.index, ib.term))
        oc.appresp_sequential(n, G, (want["group"], want["flags"], want["index"], want["term"]),
                              st, threads=8)
    assert np.array_equal(u64(tr.match), st["match"])
    assert np.array_equal(u64(tr.committed), st["committed"])
    assert np.array_equal(tr.active.cpu().numpy().view(np.uint16)[:G], st["active"])
    sd = tr.stepdown_at.cpu().numpy().view(np.uint32)
    assert np.array_equal(sd != 0xFFFFFFFF, st["stepped_down"] != 0)
    assert int((st["committed"] > 0).sum()) > G // 2  # commits advanced
