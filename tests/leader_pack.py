"""Packing between the oracle's LeaderGroup objects and the engine's SoA
arrays (etcd_amd.quorum.leader), plus a seeded random-state generator for
parity fuzzing.  Test infrastructure."""
from __future__ import annotations

import numpy as np

from oracle import leader_ref as L

MAX_RUNS = 8


def pack(groups, inflight_cap: int, readq_cap: int):
    G = len(groups)
    off = np.zeros(G + 1, np.uint32)
    for i, g in enumerate(groups):
        off[i + 1] = off[i] + g.n_slots
    S = int(off[-1])
    a = {
        "off": off, "cfg": np.zeros(G, np.uint32), "meta": np.zeros(G, np.uint32),
        "term": np.zeros(G, np.uint64), "committed": np.zeros(G, np.uint64),
        "first_index": np.zeros(G, np.uint64), "last_index": np.zeros(G, np.uint64),
        "snap_index": np.zeros(G, np.uint64), "snap_term": np.zeros(G, np.uint64),
        "max_ents": np.zeros(G, np.uint64),
        "run_start": np.zeros(G * MAX_RUNS, np.uint64), "run_term": np.zeros(G * MAX_RUNS, np.uint64),
        "match": np.zeros(S, np.uint64), "next": np.zeros(S, np.uint64),
        "pending_snapshot": np.zeros(S, np.uint64), "pstate": np.zeros(S, np.uint8),
        "infl_pos": np.zeros(S, np.uint32), "infl_buf": np.zeros(S * inflight_cap, np.uint64),
        "rq_ctx": np.zeros(G * readq_cap, np.uint64), "rq_index": np.zeros(G * readq_cap, np.uint64),
        "rq_meta": np.zeros(G * readq_cap, np.uint32),
    }
    for i, g in enumerate(groups):
        a["cfg"][i] = g.mask_in | (g.mask_out << 16)
        assert 1 <= len(g.log.runs) <= MAX_RUNS and len(g.readq) <= readq_cap
        a["meta"][i] = (g.leader_slot | (g.transferee << 8) | (len(g.log.runs) << 16)
                        | (len(g.readq) << 20) | ((1 << 25) if g.pending_readindex else 0))
        a["term"][i] = g.term
        a["committed"][i] = g.log.committed
        a["first_index"][i] = g.log.first
        a["last_index"][i] = g.log.last
        a["snap_index"][i] = g.log.snap_index
        a["snap_term"][i] = g.log.snap_term
        a["max_ents"][i] = g.log.max_ents
        for r, (st, t) in enumerate(g.log.runs):
            a["run_start"][r * G + i] = st  # run-major
            a["run_term"][r * G + i] = t
        for j, p in enumerate(g.prs):
            s = int(off[i]) + j
            a["match"][s] = p.match
            a["next"][s] = p.next
            a["pending_snapshot"][s] = p.pending_snapshot
            a["pstate"][s] = p.state | (4 if p.probe_sent else 0) | (8 if p.recent_active else 0)
            assert p.inflights.size == inflight_cap
            a["infl_pos"][s] = p.inflights.start | (p.inflights.count << 16)
            a["infl_buf"][s * inflight_cap:(s + 1) * inflight_cap] = p.inflights.buffer
        for k, rs in enumerate(g.readq):
            q = i * readq_cap + k
            a["rq_ctx"][q] = rs.ctx
            a["rq_index"][q] = rs.index
            acks = 0
            for s_ in rs.acks:
                acks |= 1 << s_
            a["rq_meta"][q] = acks | (rs.from_slot << 16)
    return a


def unpack_into(groups, a, inflight_cap: int, readq_cap: int):
    """Overwrite the mutable state of ``groups`` from engine arrays."""
    off = a["off"]
    for i, g in enumerate(groups):
        meta = int(a["meta"][i])
        g.log.committed = int(a["committed"][i])
        g.pending_readindex = bool(meta & (1 << 25))
        for j, p in enumerate(g.prs):
            s = int(off[i]) + j
            p.match = int(a["match"][s])
            p.next = int(a["next"][s])
            p.pending_snapshot = int(a["pending_snapshot"][s])
            st = int(a["pstate"][s])
            p.state, p.probe_sent, p.recent_active = st & 3, bool(st & 4), bool(st & 8)
            pos = int(a["infl_pos"][s])
            p.inflights = L.Inflights(inflight_cap, pos & 0xFFFF, pos >> 16,
                                      [int(x) for x in a["infl_buf"][s * inflight_cap:(s + 1) * inflight_cap]])
        n = (meta >> 20) & 0x1F
        q0 = i * readq_cap
        g.readq = []
        for k in range(n):
            m = int(a["rq_meta"][q0 + k])
            g.readq.append(L.ReadIndexStatus(int(a["rq_ctx"][q0 + k]), int(a["rq_index"][q0 + k]),
                                             {s_ for s_ in range(16) if (m >> s_) & 1}, m >> 16))


def state_key(g: L.LeaderGroup):
    """Everything observable about a group after a step."""
    return (g.log.committed, g.pending_readindex,
            tuple((p.match, p.next, p.pending_snapshot, p.state, p.probe_sent, p.recent_active,
                   tuple(p.inflights.fifo()), p.inflights.start) for p in g.prs),
            tuple((r.ctx, r.index, tuple(sorted(r.acks)), r.from_slot) for r in g.readq))


# --------------------------------------------------------------- fuzzing ---

def random_groups(rng: np.random.Generator, G: int, inflight_cap: int, readq_cap: int,
                  max_slots: int = 9, term_base: int = 0):
    groups = []
    for _ in range(G):
        ns = int(rng.integers(1, max_slots + 1))
        leader = int(rng.integers(0, ns))
        vin = leader_mask = 1 << leader
        for s in range(ns):
            if rng.random() < 0.75:
                vin |= 1 << s
        mout = 0
        if rng.random() < 0.2:
            for s in range(ns):
                if rng.random() < 0.5:
                    mout |= 1 << s
        del leader_mask
        term = int(rng.integers(1, 50)) + term_base
        first = int(rng.integers(1, 40))
        last = first - 1 + int(rng.integers(0, 60))
        # term runs over [first-1, last]: ascending starts, the leader's term last
        nruns = int(rng.integers(1, MAX_RUNS + 1))
        starts = sorted(set([first - 1] + [int(x) for x in rng.integers(first - 1, last + 2, nruns - 1)]))
        terms = sorted(int(x) for x in rng.integers(0, term + 1, len(starts)))
        if rng.random() < 0.8:
            terms[-1] = term
        if rng.random() < 0.1 and starts[0] > 0:
            starts[0] -= 1  # a run starting before the dummy entry
        runs = list(zip(starts, terms))
        committed = int(rng.integers(max(0, first - 1), last + 1)) if last >= first - 1 else 0
        snap = 0 if rng.random() < 0.15 else first - 1
        snap_term = terms[0]
        max_ents = int(rng.choice([1, 2, 3, 5, 1 << 62]))
        log = L.LogView(first, last, committed, runs, snap, snap_term, max_ents)
        prs = []
        for s in range(ns):
            infl = L.Inflights(inflight_cap)
            state = int(rng.choice([0, 0, 1, 1, 1, 2]))
            match = int(rng.integers(0, last + 2))
            if s == leader:
                match, state = last, 1
            nxt = match + 1 + int(rng.integers(0, 6))
            if rng.random() < 0.1:
                nxt = int(rng.integers(0, max(1, match + 1)))
            psnap = int(rng.integers(0, last + 5)) if state == 2 else int(rng.integers(0, 3) == 0) * int(rng.integers(0, 20))
            if state == 1:
                cnt = int(rng.integers(0, inflight_cap + 1))
                infl.start = int(rng.integers(0, inflight_cap))
                v = match
                for _ in range(cnt):
                    v += int(rng.integers(0, 4))
                    infl.add(v)
            prs.append(L.Progress(match=match, next=nxt, state=state, pending_snapshot=psnap,
                                  recent_active=bool(rng.random() < 0.5),
                                  probe_sent=bool(rng.random() < 0.4), inflights=infl))
        readq = []
        nq = int(rng.integers(0, readq_cap + 1)) if readq_cap else 0
        for k in range(nq):
            acks = {leader} | {s for s in range(ns) if rng.random() < 0.3}
            frm = int(rng.choice([L.NO_SLOT, leader, int(rng.integers(0, ns))]))
            readq.append(L.ReadIndexStatus(1000 + k * 7 + int(rng.integers(0, 3)) * 0, committed, acks, frm))
        transferee = int(rng.integers(0, ns)) if rng.random() < 0.2 else L.NO_SLOT
        groups.append(L.LeaderGroup(ns, vin, mout, term, leader, log, prs, transferee=transferee,
                                    readq=readq, pending_readindex=bool(rng.random() < 0.2)))
    return groups


def random_records(rng: np.random.Generator, groups, M: int, bad_frac: float = 0.01,
                   hot_groups: int = 0, hot_frac: float = 0.0):
    """M random inbox records; with hot_groups, a hot_frac share of them goes
    to the first hot_groups groups (long per-group runs, crowded chunks)."""
    G = len(groups)
    recs = []
    for _ in range(M):
        gi = int(rng.integers(0, G))
        if hot_groups and rng.random() < hot_frac:
            gi = int(rng.integers(0, hot_groups))
        if rng.random() < bad_frac:
            recs.append((G + int(rng.integers(0, 5)), L.Inbound(0, 0, 1, 1)))
            continue
        g = groups[gi]
        slot = min(15, int(rng.integers(0, g.n_slots + (1 if rng.random() < 0.05 else 0))))  # 4-bit slot field
        kind = int(rng.choice([0, 0, 0, 0, 1, 1, 2, 3]))
        r = rng.random()
        term = g.term if r < 0.85 else (g.term - 1 if r < 0.92 else (0 if r < 0.96 else g.term + 1))
        if kind in (2, 3):
            term = 0
        pr = g.prs[slot] if slot < g.n_slots else None
        base = pr.next - 1 if pr is not None else 0
        reject = bool(rng.random() < 0.3) if kind in (0, 2) else False
        if kind == 0:
            index = max(0, base + int(rng.integers(-3, 8)))
        elif kind == 1:
            index = int(rng.choice([0] + [q.ctx for q in g.readq] + [999999]))
        else:
            index = 0
        hint = max(0, index - int(rng.integers(0, 5)))
        log_term = int(rng.integers(0, g.term + 2)) if rng.random() < 0.5 else 0
        recs.append((gi, L.Inbound(kind, slot, term, index, reject, hint, log_term)))
    return recs


def records_arrays(recs):
    M = len(recs)
    group = np.array([g for g, _ in recs], np.uint32)
    slot = np.array([m.slot for _, m in recs], np.uint8)
    kind = np.array([m.kind for _, m in recs], np.uint8)
    index = np.array([m.index for _, m in recs], np.uint64)
    term = np.array([m.term for _, m in recs], np.uint64)
    reject = np.array([m.reject for _, m in recs], bool)
    hint = np.array([m.hint for _, m in recs], np.uint64)
    log_term = np.array([m.log_term for _, m in recs], np.uint64)
    return dict(group=group, slot=slot, kind=kind, index=index, term=term, reject=reject,
                hint=hint, log_term=log_term) if M else None
