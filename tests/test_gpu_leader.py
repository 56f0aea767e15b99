"""GPU parity of the leader inbox step (qb_dev_leader_step) against the
sequential CPU oracle (oracle/leader_ref.py): the reference's own scenarios
(tests/golden/leader_tables.json) replayed on the device, and seeded random
batches compared field by field (state, messages, flags, counters)."""
import copy

import numpy as np
import pytest

from oracle import leader_ref as L
from tests import leader_pack as LP
from tests import leader_scenarios as LS

pytestmark = pytest.mark.gpu

TABLES = LS.load_tables()


def _engine(groups, inflight_cap, readq_cap, read_only=0):
    from etcd_amd.quorum.leader import LeaderGroups
    return LeaderGroups(LP.pack(groups, inflight_cap, readq_cap), inflight_cap, readq_cap,
                        read_only, device="cuda")


def _inbox(recs):
    from etcd_amd.quorum.leader import LeaderInbox
    a = LP.records_arrays(recs)
    if a is None:
        return LeaderInbox.from_numpy([], [], [], [], [], device="cuda")
    return LeaderInbox.from_numpy(a["group"], a["slot"], a["kind"], a["index"], a["term"],
                                  a["reject"], a["hint"], a["log_term"], device="cuda")


def _dev_msgs(res):
    return [(int(m["group"]), int(m["type"]), int(m["to"]), int(m["index"]), int(m["log_term"]),
             int(m["commit"]), int(m["aux"])) for m in res.msgs]


def _orc_msgs(groups):
    out = []
    for gi, g in enumerate(groups):
        out += [(gi,) + m.key() for m in g.msgs]
    return out


@pytest.mark.parametrize("sc", TABLES["scenarios"], ids=[s["name"] for s in TABLES["scenarios"]])
def test_reference_scenarios_on_device(sc):
    g = LS.build_group(sc)
    cap = sc["infl_size"]
    for k, op in enumerate(sc["ops"]):
        where = f"{sc['name']} op{k}"
        if op["op"] == "propose":  # host-side op between device batches
            g.msgs = []
            g.propose(op["n"])
            LS.check_expect(where, op["expect"], [LS.msg_dict(m) for m in g.msgs], g)
            continue
        batch = [LS.inbound(m) for m in op["msgs"]] if op["op"] == "recv_batch" else [LS.inbound(op)]
        twin = copy.deepcopy(g)  # the oracle's run of the same records
        twin.msgs = []
        for j, m in enumerate(batch):
            twin.step(m, j)
        eng = _engine([g], cap, max(1, len(g.readq)))
        res = eng.step(_inbox([(0, m) for m in batch]))
        LP.unpack_into([g], eng.numpy(), cap, max(1, len(g.readq)))
        msgs = [dict(zip(LS.MSG_FIELDS, m[1:])) for m in _dev_msgs(res)]
        LS.check_expect(where, op["expect"], msgs, g)
        assert [tuple(m.values()) for m in msgs] == [m.key() for m in twin.msgs], where
        assert LP.state_key(g) == LP.state_key(twin), where


def _split_reads(om):
    """The oracle's messages with its local ReadStates (type 255) taken out
    into (group, index, ctx) — the outbox's read_states form."""
    return ([m for m in om if m[1] != 255], [(m[0], m[3], m[6]) for m in om if m[1] == 255])


def _dev_reads(res):
    G = len(res.read_off) - 1
    grp = np.repeat(np.arange(G), np.diff(res.read_off))
    return [(int(g), int(r["index"]), int(r["ctx"])) for g, r in zip(grp, res.read_states)]


def _fuzz(seed, G, M, inflight_cap, readq_cap, read_only=0, max_slots=9, hot_groups=0,
          hot_frac=0.0, term_base=0, options=0, outbox=False, read_states=False):
    rng = np.random.default_rng(seed)
    groups = LP.random_groups(rng, G, inflight_cap, readq_cap, max_slots, term_base)
    for g in groups:
        g.read_only = read_only
    recs = LP.random_records(rng, groups, M, hot_groups=hot_groups, hot_frac=hot_frac)
    eng = _engine(groups, inflight_cap, readq_cap, read_only)
    eng.options = options
    if read_states:
        res = eng.step_outbox(_inbox(recs), read_states=True)
    else:
        res = eng.step_outbox(_inbox(recs)) if outbox else eng.step(_inbox(recs))
    orc = copy.deepcopy(groups)
    for g in orc:
        g.msgs = []
    stats = L.run_batch(orc, recs)
    dev = copy.deepcopy(groups)
    LP.unpack_into(dev, eng.numpy(), inflight_cap, readq_cap)
    for gi in range(G):
        assert LP.state_key(dev[gi]) == LP.state_key(orc[gi]), f"seed {seed} group {gi}"
    om = _orc_msgs(orc)
    if read_states:
        om, reads = _split_reads(om)
        assert reads, "the case releases no local read"
        assert _dev_reads(res) == reads
    assert res.msg_total == len(om)
    assert _dev_msgs(res) == om
    want_sd = np.array([0xFFFFFFFF if g.stepped_down_at is None else g.stepped_down_at for g in orc],
                       np.uint32)
    assert np.array_equal(res.stepdown_at, want_sd)
    want_fl = np.array([(1 if g.advanced else 0) | (2 if g.released_pending else 0)
                        | (4 if g.stepped_down_at is not None else 0) for g in orc], np.uint8)
    assert np.array_equal(res.gflags, want_fl)
    assert res.stats["applied"] == stats["applied"]
    assert res.stats["stale_term"] == stats["stale"]
    assert res.stats["higher_term"] == stats["higher"]
    assert res.stats["non_member"] == stats["nonmember"]
    assert res.stats["after_stepdown"] == stats["after"]
    assert res.stats["bad_group"] == stats["bad"]
    assert res.stats["msgs"] == len(om) and res.stats["msgs_dropped"] == 0


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_small(seed):
    _fuzz(seed, G=400, M=1500, inflight_cap=3, readq_cap=4)


def test_fuzz_lease_based_and_wide():
    _fuzz(11, G=300, M=1200, inflight_cap=5, readq_cap=2, read_only=1, max_slots=16)


def test_fuzz_terms_past_32_bits():
    """Group, record and log terms straddling 2^32 - 1: the bucketing moves
    the term as u32 with an escape to the original batch (qb_bucket.h)."""
    _fuzz(51, G=3000, M=9000, inflight_cap=6, readq_cap=3, term_base=(1 << 32) - 25)


@pytest.mark.parametrize("cap", [1, 2, 600])
def test_fuzz_ring_capacities(cap):
    """MaxInflightMsgs at its small end (a one-entry ring: full after every
    send) and far past the others (600), both output forms."""
    _fuzz(60 + cap, G=200, M=900, inflight_cap=cap, readq_cap=2)
    _fuzz(70 + cap, G=200, M=900, inflight_cap=cap, readq_cap=2, outbox=True)


def test_fuzz_larger():
    _fuzz(21, G=5000, M=12000, inflight_cap=8, readq_cap=4)


def test_fuzz_long_runs():
    """Groups with ~100 records in one batch (runs ordered outside LDS),
    chunks still placed through LDS."""
    _fuzz(41, G=600, M=2000, inflight_cap=6, readq_cap=3, hot_groups=2, hot_frac=0.1)


def test_fuzz_crowded_chunk():
    """A chunk with more records than the LDS placement holds (> 1536)."""
    _fuzz(42, G=300, M=5000, inflight_cap=6, readq_cap=3, hot_groups=3, hot_frac=0.5)


def test_fuzz_atomic_grouping():
    """The grouping used beyond the bucket geometry (> 134M groups per
    shard): per-record global atomics, then the same gather and step
    (QB_LEADER_OPT_ATOMIC_GROUPING)."""
    _fuzz(31, G=3000, M=9000, inflight_cap=6, readq_cap=3, max_slots=16, options=1)


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzz_outbox(seed):
    """qb_dev_leader_step_outbox: the same step with the messages left in the
    per-group outbox (8 k-major slots + overflow chunks), read back in group
    order — identical to the oracle (and so to qb_dev_leader_step)."""
    _fuzz(seed, G=400, M=1500, inflight_cap=3, readq_cap=4, outbox=True)


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzz_outbox_read_states(seed):
    """The outbox's ReadState area: the local reads' answers leave the
    messages (raft.go:1737-1745 appends them to r.readStates), in release
    order per group; every other message, the state and the flags as the
    oracle's."""
    _fuzz(seed, G=400, M=1500, inflight_cap=3, readq_cap=4, read_states=True)
    _fuzz(seed + 10, G=300, M=5000, inflight_cap=6, readq_cap=16, hot_groups=3, hot_frac=0.5,
          read_states=True)


def test_fuzz_outbox_overflow_chunks():
    """Hot groups emit far more than 8 messages in one batch: the outbox's
    overflow chains (32-message chunks) hold the rest, in emission order."""
    _fuzz(41, G=600, M=2000, inflight_cap=6, readq_cap=3, hot_groups=2, hot_frac=0.1, outbox=True)
    _fuzz(42, G=300, M=5000, inflight_cap=6, readq_cap=3, hot_groups=3, hot_frac=0.5, outbox=True)


def test_outbox_without_chunks_keeps_eight_per_group():
    """nchunks = 0: a group keeps its first 8 messages and the rest is
    counted as dropped (QB_LSTAT_MSGS_DROPPED), every other output exact."""
    rng = np.random.default_rng(43)
    groups = LP.random_groups(rng, 300, 6, 3, 9, 0)
    recs = LP.random_records(rng, groups, 5000, hot_groups=3, hot_frac=0.5)
    eng = _engine(groups, 6, 3)
    res = eng.step_outbox(_inbox(recs), nchunks=0)
    orc = copy.deepcopy(groups)
    for g in orc:
        g.msgs = []
    L.run_batch(orc, recs)
    want = []
    for gi, g in enumerate(orc):
        want += [(gi,) + m.key() for m in g.msgs[:8]]
    assert _dev_msgs(res) == want
    total = sum(len(g.msgs) for g in orc)
    assert total > len(want)
    assert res.stats["msgs"] == total and res.stats["msgs_dropped"] == total - len(want)


def test_empty_batch_and_truncated_output():
    rng = np.random.default_rng(5)
    groups = LP.random_groups(rng, 50, 4, 2)
    eng = _engine(groups, 4, 2)
    res = eng.step(_inbox([]))
    assert res.msg_total == 0 and res.stats["applied"] == 0
    recs = LP.random_records(rng, groups, 400, bad_frac=0)
    orc = copy.deepcopy(groups)
    for g in orc:
        g.msgs = []
    L.run_batch(orc, recs)
    om = _orc_msgs(orc)
    cap = len(om) // 2
    res = eng.step(_inbox(recs), msg_cap=cap)
    assert res.msg_total == len(om)
    assert _dev_msgs(res) == om[:cap]
    assert res.stats["msgs_dropped"] == len(om) - cap


@pytest.mark.parametrize("outbox", [False, True])
def test_streaming_workload_vs_c_oracle(outbox):
    """The bench's streaming workload at 1M groups, six consecutive batches,
    every state array and every message against the C oracle (through the
    group-ordered array and through the outbox)."""
    import torch
    from etcd_amd.quorum.leader import streaming_inbox, synth_streaming
    from tests import oracle_c as oc
    G = 1 << 20
    lg, base = synth_streaming(G, device="cuda")
    host = {k: v.copy() for k, v in lg.numpy().items()}
    for k in range(6):
        ib = streaming_inbox(G, base, k, device="cuda")
        res = lg.step_outbox(ib) if outbox else lg.step(ib, msg_cap=6 * G)
        rec = {"group": ib.group.cpu().numpy().view(np.uint32),
               "flags": ib.flags.cpu().numpy(), "index": ib.index.cpu().numpy().view(np.uint64),
               "term": ib.term.cpu().numpy().view(np.uint64),
               "hint": ib.hint.cpu().numpy().view(np.uint64),
               "log_term": ib.log_term.cpu().numpy().view(np.uint64)}
        msgs, total, sd, gf, stats = oc.leader_step(host, 32, 0, 0, rec, threads=16,
                                                    msg_cap=6 * G)
        dev = lg.numpy()
        for name in host:
            assert np.array_equal(dev[name], host[name]), f"step {k}: {name}"
        assert res.msg_total == total
        assert np.array_equal(res.msgs.view(np.uint8), msgs.view(np.uint8)), f"step {k}: msgs"
        assert np.array_equal(res.stepdown_at, sd) and np.array_equal(res.gflags, gf)
        assert res.stats["applied"] == int(stats[0]) == G
    torch.cuda.synchronize()


@pytest.mark.parametrize("outbox", [False, True])
def test_skewed_batch_overflows_reserved_regions(outbox):
    """A batch concentrated on two super-buckets (the first 65536 of 1M
    groups) plus 10 % of the rest: their runs outgrow the reserved regions
    (capacity ~2x an even share), the excess continues in the regions'
    overflow pool parts and the chunk placement reads them as extra run-table
    rows — every state array and message against the C oracle, the
    bucketing's bad-group count included."""
    import torch
    from etcd_amd.quorum.leader import LeaderInbox, streaming_inbox, synth_streaming
    from tests import oracle_c as oc
    G = 1 << 20
    lg, base = synth_streaming(G, device="cuda")
    host = {k: v.copy() for k, v in lg.numpy().items()}
    full = streaming_inbox(G, base, 0, device="cuda")
    col = {n: getattr(full, n).cpu().numpy() for n in ("group", "flags", "index", "term", "hint",
                                                       "log_term")}
    grp = col["group"].view(np.uint32)
    rng = np.random.default_rng(5)
    keep = (grp < 65536) | (rng.random(grp.size) < 0.1)
    keep[:64] = True
    grp = grp.copy()
    grp[:64] = G + 7  # a few bad groups, counted by the bucketing
    flags = col["flags"][keep]
    ib = LeaderInbox.from_numpy(grp[keep], flags & 0x0F, (flags >> 4) & 3,
                                col["index"].view(np.uint64)[keep], col["term"].view(np.uint64)[keep],
                                reject=(flags & 0x80) != 0, hint=col["hint"].view(np.uint64)[keep],
                                log_term=col["log_term"].view(np.uint64)[keep])
    M = int(keep.sum())
    assert M > 150_000
    res = lg.step_outbox(ib) if outbox else lg.step(ib, msg_cap=6 * M)
    rec = {"group": ib.group.cpu().numpy().view(np.uint32), "flags": ib.flags.cpu().numpy(),
           "index": ib.index.cpu().numpy().view(np.uint64),
           "term": ib.term.cpu().numpy().view(np.uint64),
           "hint": ib.hint.cpu().numpy().view(np.uint64),
           "log_term": ib.log_term.cpu().numpy().view(np.uint64)}
    msgs, total, sd, gf, stats = oc.leader_step(host, 32, 0, 0, rec, threads=16, msg_cap=6 * M)
    dev = lg.numpy()
    for name in host:
        assert np.array_equal(dev[name], host[name]), name
    assert res.msg_total == total
    assert np.array_equal(res.msgs.view(np.uint8), msgs.view(np.uint8))
    assert np.array_equal(res.stepdown_at, sd) and np.array_equal(res.gflags, gf)
    assert res.stats["applied"] == int(stats[0]) == M - 64
    assert res.stats["bad_group"] == 64
    torch.cuda.synchronize()


def test_dense_batch_many_run_table_rows_vs_c_oracle():
    """Eight streaming batches concatenated into one call (8 records per
    group over 1M groups): the regions hold ~32K records, so a chunk's run
    table has more than 64 rows (k_ld_chunk_runs<true>) — every state array
    and message against the C oracle on the same batch."""
    import torch
    from etcd_amd.quorum.leader import LeaderInbox, streaming_inbox, synth_streaming
    from tests import oracle_c as oc
    G = 1 << 20
    lg, base = synth_streaming(G, device="cuda")
    host = {k: v.copy() for k, v in lg.numpy().items()}
    parts = [streaming_inbox(G, base, k, device="cuda") for k in range(8)]
    col = {n: torch.cat([getattr(p_, n) for p_ in parts]).cpu().numpy()
           for n in ("group", "flags", "index", "term", "hint", "log_term")}
    flags = col["flags"]
    ib = LeaderInbox.from_numpy(col["group"].view(np.uint32), flags & 0x0F, (flags >> 4) & 3,
                                col["index"].view(np.uint64), col["term"].view(np.uint64),
                                reject=(flags & 0x80) != 0, hint=col["hint"].view(np.uint64),
                                log_term=col["log_term"].view(np.uint64))
    M = 8 * G
    res = lg.step(ib, msg_cap=6 * M)
    rec = {"group": ib.group.cpu().numpy().view(np.uint32), "flags": ib.flags.cpu().numpy(),
           "index": ib.index.cpu().numpy().view(np.uint64),
           "term": ib.term.cpu().numpy().view(np.uint64),
           "hint": ib.hint.cpu().numpy().view(np.uint64),
           "log_term": ib.log_term.cpu().numpy().view(np.uint64)}
    msgs, total, sd, gf, stats = oc.leader_step(host, 32, 0, 0, rec, threads=16, msg_cap=6 * M)
    dev = lg.numpy()
    for name in host:
        assert np.array_equal(dev[name], host[name]), name
    assert res.msg_total == total
    assert np.array_equal(res.msgs.view(np.uint8), msgs.view(np.uint8))
    assert np.array_equal(res.stepdown_at, sd) and np.array_equal(res.gflags, gf)
    assert res.stats["applied"] == int(stats[0]) == M
    torch.cuda.synchronize()


@pytest.mark.timeout(600)
def test_dense_batch_overflow_pool_windows_vs_c_oracle():
    """64 streaming batches concatenated into one call over 64K groups (64
    records per group, 4M records): every region receives about twice its
    capacity (which the run table's 256 rows bound), so each region's excess
    continues in ~32 overflow pool parts and a chunk reads ~256 pool rows in
    four 64-row windows.  ADVICE r4: the round-4 overflow area was scanned
    whole by every flagged chunk (quadratic: 256 chunks x 2M overflow
    records here); the pool keeps the step linear — timed, and every state
    array and message against the C oracle."""
    import time

    import torch
    from etcd_amd.quorum.leader import LeaderInbox, streaming_inbox, synth_streaming
    from tests import oracle_c as oc
    G, R = 1 << 16, 64
    lg, base = synth_streaming(G, device="cuda")
    host = {k: v.copy() for k, v in lg.numpy().items()}
    parts = [streaming_inbox(G, base, k, device="cuda") for k in range(R)]
    cols = {n: torch.cat([getattr(p_, n) for p_ in parts]) for n in
            ("group", "flags", "index", "term", "hint", "log_term")}
    del parts
    ib = LeaderInbox(**{n: cols[n] for n in ("group", "flags", "index", "term", "hint",
                                             "log_term")})
    M = R * G
    ib._m = M
    nchunks = M // 8 + 1024
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ob, st = lg.step_outbox(ib, nchunks=nchunks, fetch=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert dt < 2.0, f"leader step over {M} records took {dt:.2f} s"
    res = lg.fetch_outbox(ob, st, nchunks)
    rec = {n: cols[n].cpu().numpy() for n in cols}
    rec = {"group": rec["group"].view(np.uint32), "flags": rec["flags"],
           "index": rec["index"].view(np.uint64), "term": rec["term"].view(np.uint64),
           "hint": rec["hint"].view(np.uint64), "log_term": rec["log_term"].view(np.uint64)}
    msgs, total, sd, gf, stats = oc.leader_step(host, 32, 0, 0, rec, threads=16,
                                                msg_cap=res.msg_total + 1)
    dev = lg.numpy()
    for name in host:
        assert np.array_equal(dev[name], host[name]), name
    assert res.msg_total == total
    assert np.array_equal(res.msgs.view(np.uint8), msgs.view(np.uint8))
    assert np.array_equal(res.stepdown_at, sd) and np.array_equal(res.gflags, gf)
    assert res.stats["applied"] == int(stats[0]) == M
    torch.cuda.synchronize()


@pytest.mark.parametrize("outbox", [False, True, "read_states"])
def test_readindex_workload_vs_c_oracle(outbox):
    """The ReadIndex bench workload (§8f row 2) at 256K groups: queues,
    released reads and every message against the C oracle (read_states: the
    outbox's ReadState area holds the local answers)."""
    from etcd_amd.quorum.leader import readindex_inbox, synth_readindex
    from tests import oracle_c as oc
    G, Q = 1 << 18, 4
    lg, last_ctx, _ = synth_readindex(G, Q, device="cuda")
    host = {k: v.copy() for k, v in lg.numpy().items()}
    ib = readindex_inbox(G, last_ctx, device="cuda")
    if outbox == "read_states":
        res = lg.step_outbox(ib, read_states=True)
    else:
        res = lg.step_outbox(ib) if outbox else lg.step(ib, msg_cap=8 * G)
    rec = {"group": ib.group.cpu().numpy().view(np.uint32), "flags": ib.flags.cpu().numpy(),
           "index": ib.index.cpu().numpy().view(np.uint64),
           "term": ib.term.cpu().numpy().view(np.uint64),
           "hint": ib.hint.cpu().numpy().view(np.uint64),
           "log_term": ib.log_term.cpu().numpy().view(np.uint64)}
    msgs, total, sd, gf, stats = oc.leader_step(host, lg.inflight_cap, Q, 0, rec, threads=16,
                                                msg_cap=8 * G)
    dev = lg.numpy()
    for name in host:
        assert np.array_equal(dev[name], host[name]), name
    if outbox == "read_states":
        local = msgs["type"] == 255
        assert total == Q * G and res.msg_total == int((~local).sum()) and local.any()
        assert np.array_equal(res.msgs.view(np.uint8), msgs[~local].view(np.uint8))
        assert np.array_equal(res.read_states["index"], msgs["index"][local])
        assert np.array_equal(res.read_states["ctx"], msgs["aux"][local])
        want_off = np.zeros(G + 1, np.int64)
        want_off[1:] = np.cumsum(np.bincount(msgs["group"][local], minlength=G))
        assert np.array_equal(res.read_off, want_off)
        return
    assert res.msg_total == total == Q * G
    assert np.array_equal(res.msgs.view(np.uint8), msgs.view(np.uint8))


def test_meta_counts_past_their_bounds_read_as_the_bounds():
    """A group meta word whose pending-read count exceeds readq_cap or whose
    term-run count exceeds QB_LEADER_MAX_RUNS is read as the bound (the
    header's contract): the step stays inside the caller's arrays and the
    ReadState area and gives what the bounded word gives."""
    import torch
    from etcd_amd.quorum.leader import readindex_inbox, synth_readindex
    G, Q = 4096, 4
    outs = []
    for qbits, rbits in ((Q, 8), (31, 15)):
        torch.manual_seed(7)
        lg, last_ctx, _ = synth_readindex(G, Q, device="cuda")
        m = lg.t["meta"]
        m.copy_((m & ~((0x1F << 20) | (0xF << 16))) | (qbits << 20) | (rbits << 16))
        ib = readindex_inbox(G, last_ctx, device="cuda")
        res = lg.step_outbox(ib, read_states=True)
        outs.append((res, lg.numpy()))
    (a, sa), (b, sb) = outs
    assert a.read_off[-1] > 0 and np.all(np.diff(b.read_off) <= Q)
    assert np.array_equal(a.msgs.view(np.uint8), b.msgs.view(np.uint8))
    assert np.array_equal(a.read_states.view(np.uint8), b.read_states.view(np.uint8))
    assert np.array_equal(a.read_off, b.read_off)
    for name in sa:
        x, y = sa[name], sb[name]
        if name == "meta":  # the count bits of an untouched group stay as written
            qx, qy = (x >> 20) & 0x1F, np.minimum((y >> 20) & 0x1F, Q)
            assert np.array_equal(qx, qy), "meta: pending reads"
            keep = np.array(~(0x1FF << 16) & 0xFFFFFFFF).astype(x.dtype)
            x, y = x & keep, y & keep
        assert np.array_equal(x, y), name
