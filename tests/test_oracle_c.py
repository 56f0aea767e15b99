"""The C oracle (full-size checker) against the pinned Python restatement,
and the product's host-side generator against the oracle's independent copy
of the synthetic-input spec.  CPU only."""
import random

import numpy as np
import pytest

from oracle import quorum_ref as q
from tests import oracle_c as oc


def _csr_from_groups(groups):
    """groups: list of (slot values, mask_in, mask_out, voted, granted)."""
    off = np.zeros(len(groups) + 1, np.uint32)
    vals, cfg, votes = [], np.zeros(len(groups), np.uint32), np.zeros(len(groups), np.uint32)
    for g, (v, mi, mo, vd, gr) in enumerate(groups):
        off[g + 1] = off[g] + len(v)
        vals += v
        cfg[g] = mi | (mo << 16)
        votes[g] = vd | (gr << 16)
    return off, np.asarray(vals, np.uint64), cfg, votes


def _random_groups(rng, G, big=False):
    groups = []
    for _ in range(G):
        s = rng.randrange(0, 17)
        hi = (1 << 64) - 1 if big else 20
        v = [rng.randrange(0, hi + 1) for _ in range(s)]
        full = (1 << s) - 1
        mi = rng.getrandbits(16) & full
        mo = rng.getrandbits(16) & full if rng.random() < 0.5 else 0
        vd = rng.getrandbits(16) & full
        gr = rng.getrandbits(16) & vd
        groups.append((v, mi, mo, vd, gr))
    return groups


def _py_expected(groups):
    commit, vote = [], []
    for v, mi, mo, vd, gr in groups:
        ids = list(range(1, len(v) + 1))
        c0 = {ids[j] for j in range(len(v)) if (mi >> j) & 1}
        c1 = {ids[j] for j in range(len(v)) if (mo >> j) & 1}
        acked = {ids[j]: v[j] for j in range(len(v))}
        votes = {ids[j]: bool((gr >> j) & 1) for j in range(len(v)) if (vd >> j) & 1}
        commit.append(q.joint_committed_index(c0, c1, acked))
        vote.append(q.joint_vote_result(c0, c1, votes))
    return np.asarray(commit, np.uint64), np.asarray(vote, np.uint8)


@pytest.mark.parametrize("big", [False, True])
def test_csr_eval_matches_python(big):
    rng = random.Random(7 + big)
    groups = _random_groups(rng, 3000, big)
    off, vals, cfg, votes = _csr_from_groups(groups)
    c, v = oc.csr_eval(off, vals, cfg, votes)
    ec, ev = _py_expected(groups)
    assert np.array_equal(c, ec)
    assert np.array_equal(v, ev)
    c2, v2 = oc.csr_eval(off, vals, cfg, votes, threads=4)
    assert np.array_equal(c2, ec) and np.array_equal(v2, ev)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 9, 11, 16])
def test_fixed_faithful_soa_agree(n):
    match, vd, gr, _ = oc.gen_fixed(0x5EED0002, n, 5000)
    c1, v1 = oc.fixed_eval(n, match, vd, gr)
    maps = oc.faithful_maps(n, match, vd, gr)
    c2, v2 = oc.faithful_eval(maps, 5000)
    c3, v3 = oc.faithful_eval(maps, 5000, threads=3)
    assert np.array_equal(c1, c2) and np.array_equal(v1, v2)
    assert np.array_equal(c1, c3) and np.array_equal(v1, v3)
    # spot-check against the Python restatement
    for g in range(0, 5000, 97):
        ids = set(range(1, n + 1))
        acked = {j + 1: int(match[j, g]) for j in range(n)}
        votes = {j + 1: bool((int(gr[g]) >> j) & 1) for j in range(n) if (int(vd[g]) >> j) & 1}
        assert int(c1[g]) == q.majority_committed_index(ids, acked)
        assert int(v1[g]) == q.majority_vote_result(ids, votes)


def test_generator_spec_properties():
    match, vd, gr, ts = oc.gen_fixed(0x5EED0002, 5, 200000)
    last = match[0]
    assert (last >= 1).all()
    high = last >= np.uint64(1 << 63)
    assert 0.005 < high.mean() < 0.02          # ~1% of groups above 2^63
    assert ((match[1:] == 0).mean() - 0.05) ** 2 < 1e-4  # 5% absent followers
    assert (ts <= last).all() and (ts >= 1).all()
    assert ((vd & ~np.uint8(31)) == 0).all() and ((gr & ~vd) == 0).all()


def test_csr_generator_shapes():
    off, match, cfg, votes = oc.gen_csr(0x5EED0003, "ragged", 50000)
    s = np.diff(off.astype(np.int64))
    assert s.min() >= 3 and s.max() <= 11
    mi = cfg & 0xFFFF
    n = np.array([bin(int(x)).count("1") for x in mi])
    assert n.min() >= 3 and n.max() <= 9
    assert ((cfg >> 16) == 0).all()
    assert (mi & 1).all()  # slot 0 (leader) is always a voter
    off, match, cfg, votes = oc.gen_csr(0x5EED0004, "joint", 50000)
    s = np.diff(off.astype(np.int64))
    assert s.min() >= 5 and s.max() <= 10
    for x, u in zip(cfg[:2000], s[:2000]):
        mi, mo = int(x) & 0xFFFF, int(x) >> 16
        assert bin(mi).count("1") == 5 and bin(mo).count("1") == 5
        assert bin(mi | mo).count("1") == u


def test_product_host_offsets_match_oracle():
    """qb_host_synth_* (product, C ABI host functions — no GPU needed) must
    produce the same CSR offsets as the oracle's independent spec copy."""
    from etcd_amd import _lib
    for kind, fn in (("ragged", "qb_host_synth_csr_offsets"),
                     ("joint", "qb_host_synth_joint_offsets")):
        for g_begin in (0, 123457):
            off_o, _, _, _ = oc.gen_csr(0x5EED0003, kind, 20000, g_begin)
            off_p = np.empty(20001, np.uint32)
            _lib.call(fn, 0x5EED0003, 20000, g_begin, off_p.ctypes.data)
            assert np.array_equal(off_o, off_p)


def test_sequential_appresp_matches_python():
    """orc_fixed_appresp_sequential against a direct Python restatement of
    raft.Step / stepLeader / MaybeUpdate / maybeCommit."""
    rng = random.Random(11)
    n, G, M = 5, 64, 4000
    match = np.zeros((n, G), np.uint64)
    nxt = np.ones((n, G), np.uint64)
    term = np.array([rng.randrange(2, 6) for _ in range(G)], np.uint64)
    ts = np.array([rng.randrange(1, 40) for _ in range(G)], np.uint64)
    last = np.full(G, 1000, np.uint64)
    st = {"match": match.copy(), "next": nxt.copy(), "active": np.zeros(G, np.uint16),
          "term": term, "term_start": ts, "last_index": last,
          "committed": np.zeros(G, np.uint64), "stepped_down": np.zeros(G, np.uint8)}
    group = np.array([rng.randrange(0, G + 2) for _ in range(M)], np.uint32)
    slot = np.array([rng.randrange(0, 7) for _ in range(M)], np.uint8)
    rej = np.array([rng.random() < 0.1 for _ in range(M)], bool)
    flags = (slot | (rej.astype(np.uint8) << 7)).astype(np.uint8)
    index = np.array([rng.randrange(0, 200) for _ in range(M)], np.uint64)
    rterm = np.array([int(term[g]) + rng.choice([0, 0, 0, 0, -1, 1]) if g < G else 3
                      for g in group], np.uint64)
    stats = oc.appresp_sequential(n, G, (group, flags, index, rterm), st)

    # Python restatement
    pm, pn = match.copy(), nxt.copy()
    act = [0] * G
    com = [0] * G
    down = [False] * G
    for i in range(M):
        g, s, r, idx, t = int(group[i]), int(slot[i]), bool(rej[i]), int(index[i]), int(rterm[i])
        if g >= G or s >= n or t < int(term[g]):
            continue
        if t > int(term[g]):
            down[g] = True
            continue
        if down[g]:
            continue
        act[g] |= 1 << s
        if r:
            continue
        m, nx, upd = q.progress_maybe_update(int(pm[s, g]), int(pn[s, g]), idx)
        pm[s, g], pn[s, g] = m, nx
        if upd:
            ci = q.majority_committed_index(set(range(n)), {k: int(pm[k, g]) for k in range(n)})
            com[g] = q.log_maybe_commit(com[g], ci, int(term[g]),
                                        q.window_term_of(int(ts[g]), 1000, int(term[g])))
    assert np.array_equal(st["match"], pm)
    assert np.array_equal(st["next"], pn)
    assert st["active"].tolist() == act
    assert st["committed"].tolist() == com
    assert st["stepped_down"].astype(bool).tolist() == down
    assert int(stats.sum()) == M


def _random_wide(rng, G, smax, big=True):
    off = [0]
    vals, flags = [], []
    for _ in range(G):
        s = rng.randrange(0, smax + 1)
        for _ in range(s):
            hi = (1 << 64) - 1 if big and rng.random() < 0.3 else 50
            vals.append(rng.randrange(0, hi + 1))
            f = rng.getrandbits(2)
            if rng.random() < 0.7:
                f |= 4 | (8 if rng.random() < 0.6 else 0)
            flags.append(f)
        off.append(off[-1] + s)
    return (np.asarray(off, np.uint32), np.asarray(vals, np.uint64),
            np.asarray(flags, np.uint8))


def test_wide_eval_matches_python():
    rng = random.Random(21)
    off, vals, flags = _random_wide(rng, 400, 150)
    c, v = oc.wide_eval(off, vals, flags)
    for g in range(len(off) - 1):
        a, b = int(off[g]), int(off[g + 1])
        c0 = {j for j in range(a, b) if flags[j] & 1}
        c1 = {j for j in range(a, b) if flags[j] & 2}
        acked = {j: int(vals[j]) for j in range(a, b)}
        votes = {j: bool(flags[j] & 8) for j in range(a, b) if flags[j] & 4}
        assert int(c[g]) == q.joint_committed_index(c0, c1, acked)
        assert int(v[g]) == q.joint_vote_result(c0, c1, votes)


@pytest.mark.parametrize("csr", [False, True])
@pytest.mark.parametrize("threads", [2, 7, 64])
def test_sequential_appresp_owner_partition_equals_one_thread(csr, threads):
    """The multi-thread sequential restatement (groups partitioned over
    threads, the batch stably partitioned by owner) gives exactly the
    one-thread result: state, step-downs and every stat counter, with
    duplicates, higher terms, bad groups and non-members in the batch."""
    rng = np.random.default_rng(threads * 3 + csr)
    G, M = 3001, 40000
    if csr:
        off, match, cfg, _ = oc.gen_csr(0x5EED0003, "joint", G)
        sizes = np.diff(off.astype(np.int64))
    else:
        match, _, _, _ = oc.gen_fixed(0x5EED0005, 5, G)
        sizes = np.full(G, 5)
    term = rng.integers(2, 9, size=G).astype(np.uint64)
    st = {"match": match.copy(), "active": np.zeros(G, np.uint16), "term": term,
          "term_start": np.zeros(G, np.uint64), "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    group = rng.integers(0, G + 3, size=M).astype(np.uint32)
    gg = np.minimum(group, G - 1)
    slot = (rng.integers(0, 1 << 20, size=M) % (sizes[gg] + 1)).astype(np.uint8)
    flags = (slot | ((rng.random(M) < 0.1).astype(np.uint8) << 7)).astype(np.uint8)
    index = rng.integers(0, 1 << 40, size=M).astype(np.uint64)
    rterm = (term[gg].astype(np.int64) + rng.choice([0, 0, 0, 0, -1, 1], size=M)).astype(np.uint64)
    rec = (group, flags, index, rterm)
    one = {k: v.copy() for k, v in st.items()}
    many = {k: v.copy() for k, v in st.items()}
    if csr:
        s1 = oc.csr_appresp_sequential(off, cfg, rec, one, threads=1)
        sT = oc.csr_appresp_sequential(off, cfg, rec, many, threads=threads)
    else:
        s1 = oc.appresp_sequential(5, G, rec, one, threads=1)
        sT = oc.appresp_sequential(5, G, rec, many, threads=threads)
    assert s1.tolist() == sT.tolist() and int(s1.sum()) == M
    for k in one:
        assert np.array_equal(one[k], many[k]), k


@pytest.mark.parametrize("kind", ["ragged", "joint"])
def test_faithful_joint_maps_agree_with_soa(kind):
    """The Go-map restatement of the CSR/joint form (JointConfig of two
    MajorityConfig maps, ProgressMap incl. learners, votes map) equals the
    SoA restatement on the same synthetic groups, one thread and many."""
    off, match, cfg, votes = oc.gen_csr(0x5EED0003, kind, 20000)
    c0, v0 = oc.csr_eval(off, match, cfg, votes)
    maps = oc.faithful_csr_maps(off, match, cfg, votes)
    c1, v1 = oc.faithful_joint_eval(maps, 20000)
    c2, v2 = oc.faithful_joint_eval(maps, 20000, threads=5)
    assert np.array_equal(c0, c1) and np.array_equal(v0, v1)
    assert np.array_equal(c0, c2) and np.array_equal(v0, v2)
