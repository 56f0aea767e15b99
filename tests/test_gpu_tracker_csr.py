"""GPU parity for the CSR tracker step (qb_dev_csr_tracker_step): MsgAppResp
batches over ragged voter counts, learners and joint configs — MaybeUpdate
on the slot's Progress (learners included), the non-member drop before the
term filter (node.go:356-360), step-down ordering, and maybeCommit with
JointConfig.CommittedIndex (tracker.go:162-179, joint.go:49-56) — against the
sequential one-record-at-a-time C oracle (oracle/quorum_oracle.c
appresp_range over the CSR layout)."""
import numpy as np
import pytest
import torch

from etcd_amd.quorum import batch
from tests import oracle_c as oc

pytestmark = pytest.mark.gpu
DEV = "cuda"
MAX = (1 << 64) - 1


def _state(rng, kind, G, term_base=0, seed=0x5EED0003):
    off, match, cfg, _ = oc.gen_csr(seed, kind, G)
    sizes = np.diff(off.astype(np.int64))
    last = np.zeros(G, np.uint64)
    nz = sizes > 0
    last[nz] = np.maximum.reduceat(match, off[:-1][nz].astype(np.int64)) if match.size else 0
    term = rng.integers(2, 9, size=G).astype(np.uint64) + np.uint64(term_base)
    ts = last - rng.integers(0, 128, size=G).astype(np.uint64)
    st = {"match": match.copy(), "next": (match + np.uint64(1)).copy(),
          "active": np.zeros(G, np.uint16), "term": term, "term_start": ts, "last_index": last,
          "committed": np.zeros(G, np.uint64), "stepped_down": np.zeros(G, np.uint8)}
    oc.csr_commit_all(off, cfg, st["match"], ts, st["committed"])
    return off, cfg, sizes, st


def _tracker(off, cfg, st, track_next=True, max_slots=None):
    G = len(cfg)
    tr = batch.CsrTracker(torch.from_numpy(off.view(np.int32).copy()).to(DEV),
                          torch.from_numpy(cfg.view(np.int32).copy()).to(DEV),
                          max_slots=max_slots, device=DEV, track_next=track_next)
    if st["match"].size:
        tr.match[: st["match"].size].copy_(batch.from_u64(st["match"], DEV))
        if track_next:
            tr.next[: st["match"].size].copy_(batch.from_u64(st["next"], DEV))
    act = np.zeros(G + (G & 1), np.uint16)
    act[:G] = st["active"]
    tr.active.copy_(torch.from_numpy(act.view(np.int16)))
    tr.term.copy_(batch.from_u64(st["term"], DEV))
    tr.term_start.copy_(batch.from_u64(st["term_start"], DEV))
    tr.committed.copy_(batch.from_u64(st["committed"], DEV))
    return tr


def _batch(rng, G, M, sizes, st, stale=0.01, higher=0.0, reject=0.02, nonmember=0.0, bad=0.0):
    group = rng.integers(0, G, size=M).astype(np.uint32)
    s_g = sizes[group]
    slot = (rng.integers(0, 1 << 30, size=M) % np.maximum(s_g, 1)).astype(np.uint8)
    # a group with no slots only ever gets non-member records
    slot = np.where(s_g == 0, np.uint8(0), slot).astype(np.uint8)
    if nonmember:
        past = (s_g + rng.integers(0, 3, size=M)).clip(max=15).astype(np.uint8)
        slot = np.where(rng.random(M) < nonmember, past, slot).astype(np.uint8)
    last = st["last_index"][group]
    lag = rng.integers(0, 96, size=M).astype(np.uint64)
    index = np.where(lag < last, last - lag, np.uint64(0)).astype(np.uint64)
    term = st["term"][group].copy()
    u = rng.random(M)
    term = np.where(u < stale, term - np.uint64(1), term)
    term = np.where((u >= stale) & (u < stale + higher), term + np.uint64(1), term)
    rej = rng.random(M) < reject
    if bad:
        group = np.where(rng.random(M) < bad, np.uint32(G + 3), group).astype(np.uint32)
    flags = (slot | (rej.astype(np.uint8) << 7)).astype(np.uint8)
    return group, slot, index, term.astype(np.uint64), rej, flags


def _compare(tr, st, G):
    S = st["match"].size
    assert np.array_equal(batch.as_u64(tr.match)[:S], st["match"])
    if tr.next is not None:
        assert np.array_equal(batch.as_u64(tr.next)[:S], st["next"])
    assert np.array_equal(tr.active.cpu().numpy().view(np.uint16)[:G], st["active"])
    assert np.array_equal(batch.as_u64(tr.committed), st["committed"])
    assert np.array_equal(tr.stepped_down().cpu().numpy(), st["stepped_down"].astype(bool))


CASES = [
    ("ragged", 4096, 8192, {}),
    ("ragged", 1000, 20000, {"higher": 0.002, "nonmember": 0.02, "bad": 0.01}),  # duplicates
    ("joint", 3000, 6000, {"reject": 0.2, "stale": 0.1}),
    ("joint", 5000, 30000, {"higher": 0.01, "nonmember": 0.01}),
    ("ragged", 70001, 70001, {"higher": 0.001}),                     # > 1 super-bucket
    ("joint", 1, 50, {"higher": 0.1}),
]


@pytest.mark.parametrize("kind,G,M,kw", CASES)
def test_csr_step_vs_sequential(kind, G, M, kw):
    rng = np.random.default_rng(G * 31 + M)
    off, cfg, sizes, st = _state(rng, kind, G)
    tr = _tracker(off, cfg, st)
    seq = {k: v.copy() for k, v in st.items()}
    for _ in range(3):
        group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, seq, **kw)
        stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), seq)
        tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
        _compare(tr, seq, G)
        got = tr.stats_dict()
        want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                         "bad_group", "after_stepdown"), stats.tolist()))
        assert got == want
        tr.stepdown_at.fill_(-1)   # caller re-arms the stepped-down groups
        seq["stepped_down"][:] = 0


@pytest.mark.parametrize("term_base", [20000, 0xFFFFFFFF - 5, (1 << 64) - 16])
def test_csr_step_wide_terms(term_base):
    """Group terms past the record's term field (side records) and
    straddling 2^32 - 1, where the side form ends (batch-position escapes)."""
    G = M = 20000
    rng = np.random.default_rng(term_base % 99991)
    off, cfg, sizes, st = _state(rng, "joint", G, term_base)
    tr = _tracker(off, cfg, st, track_next=False)
    st.pop("next")
    seq = {k: v.copy() for k, v in st.items()}
    for _ in range(2):
        group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, seq, stale=0.05,
                                                      higher=0.01)
        stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), seq)
        tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
        _compare(tr, seq, G)
        assert tr.stats_dict()["higher_term"] == stats[4]
        tr.stepdown_at.fill_(-1)
        seq["stepped_down"][:] = 0


def test_csr_step_learners_ack_but_never_count():
    """A learner's Progress takes the ack (MaybeUpdate, RecentActive) but the
    commit index stays the voters' quorum (tracker.go:162-179)."""
    # group 0: voters {1,2,3} + learner 4; group 1: joint {1,2,3} x {3,4,5}
    cc = batch.compile_configs([{1, 2, 3}, {1, 2, 3}], [set(), {3, 4, 5}], [{4}, set()])
    off, cfg = cc.off, cc.cfg
    st = {"match": np.array([10, 0, 0, 0, 10, 0, 0, 0, 0], np.uint64),
          "active": np.zeros(2, np.uint16), "term": np.array([5, 5], np.uint64),
          "term_start": np.array([1, 1], np.uint64), "last_index": np.array([10, 10], np.uint64),
          "committed": np.zeros(2, np.uint64), "stepped_down": np.zeros(2, np.uint8)}
    tr = _tracker(off, cfg, st, track_next=False)
    # learner (slot 3 of group 0) acks 10, voter slot 1 acks 7: commit = 7
    # group 1: slots 1, 2 ack (incoming quorum 2 of 3 at >= 8), outgoing {3,4,5}
    # (slots 2,3,4) has only slot 2 -> outgoing commit stays 0
    recs = ([0, 0, 1, 1], [3, 1, 1, 2], [10, 7, 9, 8], [5, 5, 5, 5])
    seq = {k: v.copy() for k, v in st.items()}
    flags = np.array(recs[1], np.uint8)
    oc.csr_appresp_sequential(off, cfg, (np.array(recs[0], np.uint32), flags,
                                         np.array(recs[2], np.uint64),
                                         np.array(recs[3], np.uint64)), seq)
    tr.step(batch.AppRespBatch.from_numpy(*recs, device=DEV))
    _compare(tr, seq, 2)
    assert batch.as_u64(tr.committed).tolist() == [7, 0] == seq["committed"].tolist()
    assert tr.active.cpu().numpy().view(np.uint16)[:2].tolist() == [0b1010, 0b0110]


def test_csr_empty_config_never_commits():
    """An empty config's CommittedIndex is MaxUint64 (majority.go:128-133),
    past lastIndex: raftLog.maybeCommit never commits it (log.go:328-334)."""
    off = np.array([0, 0, 2], np.uint32)
    cfg = np.array([0, 0], np.uint32)          # group 1: two learners, no voters
    st = {"match": np.array([3, 4], np.uint64), "active": np.zeros(2, np.uint16),
          "term": np.array([2, 2], np.uint64), "term_start": np.array([0, 0], np.uint64),
          "last_index": np.array([9, 9], np.uint64), "committed": np.zeros(2, np.uint64),
          "stepped_down": np.zeros(2, np.uint8)}
    tr = _tracker(off, cfg, st, track_next=False)
    adv = torch.zeros(2, dtype=torch.uint8, device=DEV)
    recs = ([0, 1, 1], [0, 1, 0], [5, 6, 7], [2, 2, 2])
    tr.step(batch.AppRespBatch.from_numpy(*recs, device=DEV), adv)
    assert batch.as_u64(tr.committed).tolist() == [0, 0]
    assert adv.cpu().tolist() == [0, 0]
    assert batch.as_u64(tr.match)[:2].tolist() == [7, 6]
    assert tr.stats_dict()["non_member"] == 1    # group 0 has no Progress at all


def test_csr_commit_table(tables):
    """TestCommit (raft/raft_test.go:1127-1174) through the CSR step with an
    empty batch, each case's voters followed by two learners holding the
    largest matches (which must not move the commit)."""
    cases = tables["TestCommit"]["cases"]
    off, match, cfg, ts = [0], [], [], []
    for c in cases:
        n = len(c["matches"])
        match += list(c["matches"]) + [1 << 40, 1 << 41]
        off.append(off[-1] + n + 2)
        cfg.append((1 << n) - 1)
        same = [i for i, t in c["log"] if t == c["term"]]
        ts.append(min(same) if same else MAX)
    G = len(cases)
    off, cfg = np.array(off, np.uint32), np.array(cfg, np.uint32)
    st = {"match": np.array(match, np.uint64), "active": np.zeros(G, np.uint16),
          "term": np.ones(G, np.uint64), "term_start": np.array(ts, np.uint64),
          "committed": np.zeros(G, np.uint64), "stepped_down": np.zeros(G, np.uint8)}
    tr = _tracker(off, cfg, st, track_next=False)
    adv = torch.zeros(G, dtype=torch.uint8, device=DEV)
    tr.commit_advance(adv)
    assert batch.as_u64(tr.committed).tolist() == [c["want"] for c in cases]
    assert adv.cpu().tolist() == [int(c["want"] > 0) for c in cases]


def test_csr_stepdown_untouched_outside_flagged_chunks():
    """stepdown_at is written only for the groups of chunks holding a
    higher-term record (quorum_batch.h): other entries keep what the caller
    left there."""
    G = M = 70001
    rng = np.random.default_rng(8)
    off, cfg, sizes, st = _state(rng, "ragged", G)
    tr = _tracker(off, cfg, st, track_next=False)
    group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, st, stale=0.0)
    hi = 12345                              # one higher-term record, group 12345
    group[7], slot[7], term[7] = hi, 0, st["term"][hi] + np.uint64(3)
    tr.stepdown_at.fill_(777)
    tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV), rearm=False)
    sd = tr.stepdown_at.cpu().numpy().view(np.uint32)
    CH = 512  # groups per K5 chunk (qb_bucket.h csr_chunk_groups)
    lo, hi_end = (hi // CH) * CH, min(G, (hi // CH + 1) * CH)
    assert sd[hi] == 7
    inside = np.arange(lo, hi_end)
    assert np.all(sd[inside[inside != hi]] == 0xFFFFFFFF)
    outside = np.ones(G, bool)
    outside[lo:hi_end] = False
    assert np.all(sd[outside] == 777)


@pytest.mark.parametrize("lo_slots,track_next", [(9, True), (14, False), (1, True)])
def test_csr_step_deferred_chunks(lo_slots, track_next):
    """Wide groups (lo_slots..16 slots, joint configs and learners): a chunk
    whose slot run is longer than the first launch's LDS buffer (8 slots per
    group) is deferred to the second launch (the table's max_slots per
    group); a higher-term record in such a chunk still sends it to the slow
    path.  Mixed widths exercise both launches in one step."""
    G, M = 5000, 20000
    rng = np.random.default_rng(lo_slots * 101 + track_next)
    sizes = rng.integers(lo_slots, 17, size=G).astype(np.int64)
    off = np.zeros(G + 1, np.uint32)
    off[1:] = np.cumsum(sizes).astype(np.uint32)
    cfg = np.zeros(G, np.uint32)
    for g in range(G):
        s = int(sizes[g])
        vin = rng.integers(1, 1 << s) & ((1 << s) - 1)
        vout = (rng.integers(1, 1 << s) & ((1 << s) - 1)) if rng.random() < 0.3 else 0
        cfg[g] = np.uint32(int(vin) | (int(vout) << 16))
    S = int(off[-1])
    last = rng.integers(1 << 20, 1 << 40, size=G).astype(np.uint64)
    match = (np.repeat(last, sizes) - rng.integers(0, 200, size=S).astype(np.uint64))
    st = {"match": match, "next": match + np.uint64(1), "active": np.zeros(G, np.uint16),
          "term": rng.integers(2, 9, size=G).astype(np.uint64),
          "term_start": last - rng.integers(0, 300, size=G).astype(np.uint64),
          "last_index": last, "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    oc.csr_commit_all(off, cfg, st["match"], st["term_start"], st["committed"])
    if not track_next:
        st.pop("next")
    tr = _tracker(off, cfg, st, track_next=track_next)
    seq = {k: v.copy() for k, v in st.items()}
    for _ in range(2):
        group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, seq, stale=0.02,
                                                      higher=0.0005, nonmember=0.01)
        stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), seq)
        tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
        _compare(tr, seq, G)
        got = tr.stats_dict()
        want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                         "bad_group", "after_stepdown"), stats.tolist()))
        assert got == want
        tr.stepdown_at.fill_(-1)
        seq["stepped_down"][:] = 0


@pytest.mark.parametrize("max_slots", [4, 8])
def test_csr_step_bound_breaking_chunk_takes_slow_path(max_slots):
    """max_slots 4 / 8 (no second K5 launch: the first launch's buffer is
    already max_slots wide): a chunk whose run is longer than its buffer —
    only a table breaking its max_slots bound has one — goes to the exact
    slow path instead of being dropped.  Voters sit in the first
    three slots and the records address slots below the bound, so the
    result is the sequential oracle's exactly."""
    CH = 512
    G, M = 4 * CH + 100, 30000
    rng = np.random.default_rng(max_slots)
    sizes = np.full(G, max_slots, np.int64)
    wide = rng.choice(CH, size=12, replace=False)          # chunk 0 breaks the bound
    sizes[wide] = max_slots + 2
    sizes[2 * CH + 5] = max_slots + 1                     # and chunk 2 (one group)
    sizes[3 * CH + 7] = 3                                 # chunk 3 stays within
    off = np.zeros(G + 1, np.uint32)
    off[1:] = np.cumsum(sizes).astype(np.uint32)
    cfg = np.full(G, 0b111, np.uint32)
    cfg[::3] = 0b111 | (0b110 << 16)                      # some joint configs
    S = int(off[-1])
    last = rng.integers(1 << 20, 1 << 40, size=G).astype(np.uint64)
    match = np.repeat(last, sizes) - rng.integers(0, 200, size=S).astype(np.uint64)
    st = {"match": match, "next": match + np.uint64(1), "active": np.zeros(G, np.uint16),
          "term": rng.integers(2, 9, size=G).astype(np.uint64),
          "term_start": last - rng.integers(0, 300, size=G).astype(np.uint64),
          "last_index": last, "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    oc.csr_commit_all(off, cfg, st["match"], st["term_start"], st["committed"])
    tr = _tracker(off, cfg, st, max_slots=max_slots)
    assert tr.max_slots == max_slots
    seq = {k: v.copy() for k, v in st.items()}
    for _ in range(2):
        bounded = np.minimum(sizes, max_slots)
        group, slot, index, term, rej, flags = _batch(rng, G, M, bounded, seq, stale=0.02)
        stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), seq)
        tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
        _compare(tr, seq, G)
        want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                         "bad_group", "after_stepdown"), stats.tolist()))
        assert tr.stats_dict() == want
        tr.stepdown_at.fill_(-1)
        seq["stepped_down"][:] = 0


@pytest.mark.timeout(300)
def test_csr_step_full_size_16m_ragged():
    """16M ragged groups (configs[2] shape) with one MsgAppResp per group."""
    G = 1 << 24
    rng = np.random.default_rng(57)
    off, cfg, sizes, st = _state(rng, "ragged", G)
    st.pop("next")
    tr = _tracker(off, cfg, st, track_next=False)
    group, slot, index, term, rej, flags = _batch(rng, G, G, sizes, st, reject=0.0,
                                                  higher=0.0001)
    oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), st, threads=16)
    tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
    assert np.array_equal(batch.as_u64(tr.match)[: st["match"].size], st["match"])
    assert np.array_equal(batch.as_u64(tr.committed), st["committed"])
    assert np.array_equal(tr.stepped_down().cpu().numpy(), st["stepped_down"].astype(bool))


@pytest.mark.parametrize("kind,G", [("ragged", 513), ("joint", 1537), ("ragged", 1)])
def test_csr_step_empty_batch_is_commit_advance(kind, G):
    """An empty batch (M = 0) through the CSR step: no record, so the state
    is unchanged except the commit advance every group gets (the step's
    maybeCommit equals commit_advance's) — here after the match rows were
    raised behind the tracker's back."""
    rng = np.random.default_rng(G)
    off, cfg, sizes, st = _state(rng, kind, G)
    tr = _tracker(off, cfg, st, track_next=False)
    bump = st["match"] + rng.integers(0, 50, size=st["match"].size).astype(np.uint64)
    tr.match[: bump.size].copy_(batch.from_u64(bump, DEV))
    want = st["committed"].copy()
    oc.csr_commit_all(off, cfg, bump, st["term_start"], want)
    adv = torch.zeros(G, dtype=torch.uint8, device=DEV)
    e = np.zeros(0)
    tr.step(batch.AppRespBatch.from_numpy(e, e, e, e, device=DEV), adv)
    assert np.array_equal(batch.as_u64(tr.committed), want)
    assert np.array_equal(batch.as_u64(tr.match)[: bump.size], bump)
    assert np.array_equal(adv.cpu().numpy().astype(bool), want != st["committed"])
    assert all(v == 0 for v in tr.stats_dict().values())


def _csr_escape_value(max_slots):
    """RecFmt for the CSR step: 512-group chunks (lgb 9), slb = 3 for a slot
    bound <= 8 else 4 — the term escape is 2047 or 1023."""
    return (1 << (23 - 9 - (3 if max_slots <= 8 else 4))) - 1


@pytest.mark.parametrize("max_slots", [4, 8, 16])
@pytest.mark.parametrize("what", ["term", "index"])
def test_csr_step_compact_record_escape_boundaries(max_slots, what):
    """ADVICE r3, CSR geometry: group terms straddling the escape value of
    the table's slot bound (packed and escaped records in one chunk), or
    record indexes straddling 2^40 with small terms; joint configs and
    learners included."""
    G, M = 3000, 9000
    E = _csr_escape_value(max_slots)
    rng = np.random.default_rng(max_slots * 7 + (what == "index"))
    lo = 1 if max_slots <= 8 else 9
    sizes = rng.integers(lo, max_slots + 1, size=G).astype(np.int64)
    off = np.zeros(G + 1, np.uint32)
    off[1:] = np.cumsum(sizes).astype(np.uint32)
    cfg = np.zeros(G, np.uint32)
    for g in range(G):
        s = int(sizes[g])
        vin = int(rng.integers(1, 1 << s)) & ((1 << s) - 1)
        vout = (int(rng.integers(1, 1 << s)) & ((1 << s) - 1)) if rng.random() < 0.3 else 0
        cfg[g] = np.uint32(vin | (vout << 16))
    S = int(off[-1])
    base = (1 << 40) - 64 if what == "index" else 1 << 30
    last = (base + rng.integers(0, 100, size=G)).astype(np.uint64)
    match = np.repeat(last, sizes) - rng.integers(0, 200, size=S).astype(np.uint64)
    term0 = E - 5 if what == "term" else 0
    st = {"match": match, "next": match + np.uint64(1), "active": np.zeros(G, np.uint16),
          "term": (rng.integers(2, 9, size=G) + term0).astype(np.uint64),
          "term_start": last - rng.integers(0, 300, size=G).astype(np.uint64),
          "last_index": last, "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    oc.csr_commit_all(off, cfg, st["match"], st["term_start"], st["committed"])
    tr = _tracker(off, cfg, st, max_slots=max_slots)
    assert tr.max_slots == max_slots
    seq = {k: v.copy() for k, v in st.items()}
    for _ in range(3):
        group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, seq, stale=0.05,
                                                      higher=0.003, nonmember=0.01)
        if what == "term":
            assert (term == E - 1).any() and (term == E).any() and (term >= E + 1).any()
        else:
            assert (index < (1 << 40)).any() and (index >= (1 << 40)).any()
        stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), seq)
        tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
        _compare(tr, seq, G)
        want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                         "bad_group", "after_stepdown"), stats.tolist()))
        assert tr.stats_dict() == want
        tr.stepdown_at.fill_(-1)
        seq["stepped_down"][:] = 0


@pytest.mark.timeout(300)
def test_csr_step_skewed_batch_overflows_reserved_regions():
    """The CSR step with a batch concentrated on one super-bucket (1.5M of 2M
    records on the groups of super-bucket 0): the regions' excess continues
    in overflow pool parts, whose chunks the first apply launch defers to
    the second (the one with the pool-window loop); the result equals the
    sequential oracle's."""
    G, M = 1 << 20, 1 << 21
    rng = np.random.default_rng(78)
    off, cfg, sizes, st = _state(rng, "ragged", G)
    st.pop("next")
    tr = _tracker(off, cfg, st, track_next=False)
    group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, st, higher=0.0005)
    hot = rng.random(M) < 0.75
    c = rng.integers(0, 128, size=M) * 8
    hg = (c * 512 + rng.integers(0, 512, size=M)).astype(np.uint32)
    group = np.where(hot, hg, group).astype(np.uint32)
    s_g = sizes[group]
    slot = (rng.integers(0, 1 << 30, size=M) % np.maximum(s_g, 1)).astype(np.uint8)
    last = st["last_index"][group]
    lag = rng.integers(0, 96, size=M).astype(np.uint64)
    index = np.where(lag < last, last - lag, np.uint64(0)).astype(np.uint64)
    term = st["term"][group].copy()
    flags = (slot | (rej.astype(np.uint8) << 7)).astype(np.uint8)
    stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), st, threads=16)
    tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
    _compare(tr, st, G)
    want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                     "bad_group", "after_stepdown"), stats.tolist()))
    assert tr.stats_dict() == want


@pytest.mark.timeout(300)
def test_csr_step_dense_batch_many_parts_per_region():
    """The CSR step with eight records per group in one call: run tables of
    more than 64 rows (see the FIXED test of the same name)."""
    G, M = 1 << 18, 1 << 21
    rng = np.random.default_rng(92)
    off, cfg, sizes, st = _state(rng, "ragged", G)
    st.pop("next")
    tr = _tracker(off, cfg, st, track_next=False)
    group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, st, higher=0.0002)
    stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), st, threads=16)
    tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
    _compare(tr, st, G)
    want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                     "bad_group", "after_stepdown"), stats.tolist()))
    assert tr.stats_dict() == want


@pytest.mark.timeout(300)
@pytest.mark.parametrize("big", [0.0, 1.0])
def test_csr_step_hot_groups_fold_in_k4(big):
    """The CSR step with hot groups (40 % of 2M records on one group, 15 % on
    eight more): K4 folds their repeated records, classing what it folds by
    the group term and, for a slot past the group's count, as non-member —
    state and every stat counter equal the sequential oracle's.  big = 1:
    every group term past the record's term field (side records, folded
    under kTermIsGroup / as term 0 by K4)."""
    G, M = 1 << 20, 1 << 21
    rng = np.random.default_rng(79 + int(big))
    off, cfg, sizes, st = _state(rng, "ragged", G)
    if big:
        st["term"] = (st["term"] + np.uint64(3000) +
                      rng.integers(0, 1 << 24, size=G).astype(np.uint64)).astype(np.uint64)
    st.pop("next")
    tr = _tracker(off, cfg, st, track_next=False)
    group, slot, index, term, rej, flags = _batch(rng, G, M, sizes, st, higher=0.0002)
    hot = rng.permutation(G)[:9].astype(np.uint32)
    u = rng.random(M)
    pick = np.where(u < 0.4, 0, np.where(u < 0.55, 1 + rng.integers(0, 8, size=M), -1))
    group = np.where(pick >= 0, hot[np.maximum(pick, 0)], group).astype(np.uint32)
    s_g = sizes[group]
    # slots up to s_g + 1: the last is no member (a non-member slot, folded too)
    slot = (rng.integers(0, 1 << 30, size=M) % (s_g + 1)).astype(np.uint8)
    last = st["last_index"][group]
    lag = rng.integers(0, 4000, size=M).astype(np.uint64)
    index = np.where(lag < last, last - lag, np.uint64(0)).astype(np.uint64)
    v = rng.random(M)
    term = st["term"][group] - (v < 0.05).astype(np.uint64)
    if big:   # a few higher terms too: their chunks take the slow path
        term = term + (v > 0.9997).astype(np.uint64)
    rej = rng.random(M) < 0.05
    flags = (slot | (rej.astype(np.uint8) << 7)).astype(np.uint8)
    stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), st, threads=16)
    tr.step(batch.AppRespBatch.from_numpy(group, slot, index, term, rej, device=DEV))
    _compare(tr, st, G)
    want = dict(zip(("applied", "rejected", "stale_term", "non_member", "higher_term",
                     "bad_group", "after_stepdown"), stats.tolist()))
    assert tr.stats_dict() == want
