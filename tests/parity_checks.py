"""Device-vs-oracle parity checks shared by the GPU tests and
``__graft_entry__.smoke()`` (test infrastructure: the oracle is the checker,
never the thing measured).  Each check runs one kernel family on the device
through the product path, the same inputs through the C / Python oracle, and
raises AssertionError naming the first difference; it returns a one-line
description (family, size, what was compared).

Reference semantics per family (paths relative to the reference's raft/):
  CommittedIndex / VoteResult      quorum/majority.go:126-210, joint.go:49-75
  MsgAppResp tracker step          raft.go:847-921, 1100-1109, 1237-1259,
                                   tracker/progress.go:144-153, log.go:328-334
  RecordVote / TallyVotes          tracker/tracker.go:252-288, raft.go:1383-1414
  QuorumActive                     tracker/tracker.go:215-225
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from etcd_amd.quorum import batch  # noqa: E402
from tests import oracle_c as oc  # noqa: E402

STAT_ORDER = ("applied", "rejected", "stale_term", "non_member", "higher_term", "bad_group",
              "after_stepdown")


def host_threads() -> int:
    import bench
    return bench.host_cpu_info()["threads"]


def check_fixed(dev, n: int, G: int, seed: int = 0x5EED0002) -> str:
    """FIXED layout (k_fixed_lds for n <= 8): CommittedIndex + VoteResult."""
    fg = batch.FixedGroups.synth(seed, n, G, device=dev)
    c, v = fg.committed_vote()
    match, vd, gr, _ = oc.gen_fixed(seed, n, G)
    ec, ev = oc.fixed_eval(n, match, vd, gr, threads=host_threads())
    assert np.array_equal(batch.as_u64(c), ec), f"fixed n={n} G={G}: CommittedIndex mismatch"
    assert np.array_equal(v.cpu().numpy(), ev), f"fixed n={n} G={G}: VoteResult mismatch"
    return f"k_fixed{'_lds' if n <= 8 else ''} {G} groups x {n} voters"


def check_csr(dev, kind: str, G: int) -> str:
    """CSR layout (k_csr): ragged voters + learners, or JointConfig 5+5."""
    seed = {"ragged": 0x5EED0003, "joint": 0x5EED0004}[kind]
    grp = batch.CsrGroups.synth(seed, kind, G, device=dev)
    c, v = grp.committed_vote()
    off, m, cfg, votes = oc.gen_csr(seed, kind, G)
    ec, ev = oc.csr_eval(off, m, cfg, votes, threads=host_threads())
    assert np.array_equal(batch.as_u64(c), ec), f"{kind} G={G}: CommittedIndex mismatch"
    assert np.array_equal(v.cpu().numpy(), ev), f"{kind} G={G}: VoteResult mismatch"
    return f"k_csr {kind} {G} groups"


def check_wide(dev, G: int = 600, smax: int = 200, seed: int = 7) -> str:
    """Groups wider than 16 slots (k_wide)."""
    from tests.test_oracle_c import _random_wide
    off, vals, flags = _random_wide(random.Random(seed), G, smax)
    d = torch.device(dev)
    grp = batch.WideGroups(torch.from_numpy(off.view(np.int32).copy()).to(d),
                           batch.from_u64(vals if vals.size else np.zeros(2, np.uint64), d),
                           torch.from_numpy(flags if flags.size else np.zeros(1, np.uint8)).to(d))
    c, v = grp.committed_vote()
    ec, ev = oc.wide_eval(off, vals, flags)
    assert np.array_equal(batch.as_u64(c), ec), "wide: CommittedIndex mismatch"
    assert np.array_equal(v.cpu().numpy(), ev), "wide: VoteResult mismatch"
    return f"k_wide {G} groups of up to {smax} slots"


def check_quorum_active(dev, G: int = 1 << 16) -> str:
    grp = batch.CsrGroups.synth(0x5EED0004, "joint", G, device=dev)
    rng = np.random.default_rng(3)
    active = rng.integers(0, 1 << 16, size=G).astype(np.uint16)
    got = grp.quorum_active(torch.from_numpy(active.view(np.int16)).to(torch.device(dev)))
    want = oc.quorum_active(grp.cfg.cpu().numpy().view(np.uint32), active)
    assert np.array_equal(got.cpu().numpy(), want), "QuorumActive mismatch"
    return f"k_quorum_active {G} joint groups"


def check_tracker_stream(dev, csr: bool, G: int, ticks: int, parity_groups: int = None,
                         stats: bool = True) -> str:
    """The bench's configs[4] stream (bench.tracker_setup: E = 64 new entries
    per tick, one record per group, 1 % stale terms) stepped tick by tick on
    the device (the bench's call: stats accumulated, stepdown_at not re-armed)
    and replayed on the sequential C oracle; after EVERY tick the state of
    the first ``parity_groups`` groups (default all) — match, committed,
    active, stepped_down — and, over all groups, every stat counter are
    compared."""
    import bench
    d = torch.device(dev)
    tr, batches, _ = bench.tracker_setup(G, ticks, 0, d, csr)
    Gs = G if parity_groups is None else min(G, parity_groups)
    off, cfg, st = bench.tracker_host_state(tr, csr, Gs)
    threads = host_threads()
    for k, b in enumerate(batches):
        tr.stats.zero_()
        tr.step(b, reset_stats=False, rearm=False)
        rec = bench.host_records(b, Gs)
        if csr:
            want = oc.csr_appresp_sequential(off, cfg, rec, st, threads=threads)
        else:
            want = oc.appresp_sequential(5, Gs, rec, st, threads=threads)
        bad = bench.tracker_state_mismatches(tr, csr, st, Gs)
        assert not bad, f"tracker{'-csr' if csr else ''} tick {k}: {bad} differ"
        if stats and Gs == G:
            got = tr.stats_dict()
            assert got == dict(zip(STAT_ORDER, (int(x) for x in want[:7]))), \
                f"tracker{'-csr' if csr else ''} tick {k}: stats {got} vs {want[:7].tolist()}"
    return (f"{'qb_dev_csr_tracker_step' if csr else 'qb_dev_fixed_tracker_step'} {G} groups x "
            f"{ticks} ticks (match, committed, active, stepdown{', stats' if stats else ''})")


def check_wire_tracker(dev, G: int = 1 << 18, ticks: int = 2) -> str:
    """The composed tick in one call (qb_dev_ingest_fixed_tracker_step) on the
    bench row's workload (tools/bench_configs.py wire_tracker_tick: encoded
    MsgAppResp, leader terms past the record's term field) against the C
    chain: the restated Message.Unmarshal (oracle/wire_oracle.c), then the
    sequential tracker oracle on its records; statuses, state and every stat
    after each tick."""
    from etcd_amd.quorum import wire
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs as bc
    d = torch.device(dev)
    n = 5
    tr, _snap, tks, rows, off, ids = bc.wire_tracker_tick(G, ticks, dev_=d)
    u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
    st = {"match": u64(tr.match).copy(), "active": tr.active.cpu().numpy().view(np.uint16)[:G].copy(),
          "term": u64(tr.term).copy(), "term_start": u64(tr.term_start).copy(),
          "committed": u64(tr.committed).copy(), "stepped_down": np.zeros(G, np.uint8)}
    h_off, h_ids = off.cpu().numpy().view(np.uint32), u64(ids)
    threads = host_threads()
    for k, (buf, nbytes, moff, grp, _direct) in enumerate(tks):
        status = wire.ingest_tracker_step(tr, buf, nbytes, moff, grp, rows=rows)
        want = oc.ingest(buf.cpu().numpy()[:nbytes], u64(moff), grp.cpu().numpy().view(np.uint32),
                         h_off, h_ids, threads=threads)
        assert np.array_equal(status.cpu().numpy(), want["status"]), f"wire-tracker tick {k}: status"
        stats = oc.appresp_sequential(n, G, (want["group"], want["flags"], want["index"],
                                             want["term"]), st, threads=threads)
        assert np.array_equal(u64(tr.match), st["match"]), f"wire-tracker tick {k}: match"
        assert np.array_equal(u64(tr.committed), st["committed"]), f"wire-tracker tick {k}: committed"
        assert np.array_equal(tr.active.cpu().numpy().view(np.uint16)[:G], st["active"]), \
            f"wire-tracker tick {k}: active"
        assert tr.stats.cpu().numpy()[:7].tolist() == [int(x) for x in stats[:7]], \
            f"wire-tracker tick {k}: stats"
    return (f"qb_dev_ingest_fixed_tracker_step {G} messages x {ticks} ticks (status, match, "
            f"committed, active, stats)")


NONE = 0xFFFFFFFF


def sequential_votes(prevote, cfg, votes0, gterm, group, flags, term):
    """The batch through one oracle Candidate per group, in batch order
    (oracle/quorum_ref.py Candidate).  Returns (votes words, stepdown_at,
    decided_at, stats[8]) as qb_dev_record_votes reports them."""
    from oracle import quorum_ref as q

    def slots(mask):
        return {s for s in range(16) if (mask >> s) & 1}
    G = len(cfg)
    cands = {}
    sd = np.full(G, NONE, np.uint32)
    dec = np.full(G, NONE, np.uint32)
    stats = np.zeros(8, np.uint64)
    for i in range(len(group)):
        g = int(group[i])
        if g >= G:
            stats[q.STAT_BAD] += 1
            continue
        c = cands.get(g)
        if c is None:
            w = int(votes0[g])
            vd, gr = w & 0xFFFF, (w >> 16) & w
            pre = {j: bool((gr >> j) & 1) for j in range(16) if (vd >> j) & 1}
            c = cands[g] = q.Candidate(prevote, int(gterm[g]), slots(int(cfg[g]) & 0xFFFF),
                                       slots(int(cfg[g]) >> 16), pre)
        was = c.decided
        st = c.step(int(flags[i]) & 0x0F, bool(flags[i] & 0x80), int(term[i]))
        stats[st] += 1
        if st == q.STAT_HIGHER:
            sd[g] = i
        if c.decided and not was:
            dec[g] = i
    out = np.asarray(votes0, np.uint32).copy()
    for g, c in cands.items():
        vd = sum(1 << j for j in c.votes)
        gr = sum(1 << j for j, v in c.votes.items() if v)
        out[g] = vd | (gr << 16)
    return out, sd, dec, stats


def check_votes(dev, prevote: bool, G: int = 500, M: int = 3000, seed: int = 1,
                p_dup: float = 0.3) -> str:
    """One vote batch (qb_dev_record_votes) against the sequential candidate,
    then TallyVotes (qb_dev_csr_tally_votes) against the oracle's tally."""
    from oracle import quorum_ref as q
    d = torch.device(dev)
    rng = np.random.default_rng(seed)
    grp = batch.CsrGroups.synth(0x5EED0007, "joint" if seed % 2 else "ragged", G, device=d)
    off = grp.off.cpu().numpy().view(np.uint32)
    cfg = grp.cfg.cpu().numpy().view(np.uint32)
    votes0 = np.zeros(G, np.uint32)
    for g in range(G):
        s = int(off[g + 1] - off[g])
        vd = gr = 0
        for j in range(s):
            if rng.random() < 0.1:
                vd |= 1 << j
                if rng.random() < 0.5:
                    gr |= 1 << j
        votes0[g] = vd | (gr << 16)
    grp.votes.copy_(torch.from_numpy(votes0.view(np.int32)))
    gterm = rng.integers(3, 9, size=G).astype(np.uint64)
    group = rng.integers(0, G + 3, size=M).astype(np.uint32)  # a few bad groups
    sizes = np.diff(off.astype(np.int64))
    gg = np.minimum(group, G - 1)
    slot = (rng.integers(0, 1 << 30, size=M) % np.maximum(sizes[gg], 1)).astype(np.uint8)
    for i in range(1, M):  # duplicates: repeat earlier (group, slot) pairs
        if rng.random() < p_dup:
            j = rng.integers(0, i)
            group[i], slot[i] = group[j], slot[j]
    reject = rng.random(M) < 0.4
    dt = rng.choice([-1, 0, 0, 0, 0, 0, 1, 2], size=M)
    term = np.where(group < G, gterm[gg].astype(np.int64) + dt, 5).astype(np.uint64)
    flags = (slot | (reject.astype(np.uint8) << 7)).astype(np.uint8)
    want_votes, want_sd, want_dec, want_stats = sequential_votes(prevote, cfg, votes0, gterm,
                                                                 group, flags, term)
    b = batch.AppRespBatch.from_numpy(group, slot, np.zeros(M, np.uint64), term, reject, device=d)
    sd, dec, gst = grp.record_votes(b, batch.from_u64(gterm, d), prevote=prevote)
    assert np.array_equal(grp.votes.cpu().numpy().view(np.uint32), want_votes), "votes words"
    assert np.array_equal(sd.cpu().numpy().view(np.uint32), want_sd), "stepdown_at"
    assert np.array_equal(dec.cpu().numpy().view(np.uint32), want_dec), "decided_at"
    assert gst.cpu().numpy().view(np.uint64).tolist() == want_stats.tolist(), "vote stats"
    gr_, rj_, res = grp.tally_votes()
    gr_, rj_, res = gr_.cpu().numpy(), rj_.cpu().numpy(), res.cpu().numpy()
    for g in range(G):
        w = int(want_votes[g])
        pre = {j: bool((w >> (16 + j)) & 1) for j in range(16) if (w >> j) & 1}
        eg, er, eres = q.tally_votes_slots(int(cfg[g]) & 0xFFFF, int(cfg[g]) >> 16, pre)
        assert (gr_[g], rj_[g], res[g]) == (eg, er, eres), f"tally of group {g}"
    return (f"qb_dev_record_votes ({'pre-vote' if prevote else 'vote'}) {M} responses over {G} "
            f"groups + qb_dev_csr_tally_votes")
