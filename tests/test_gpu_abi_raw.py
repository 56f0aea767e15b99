"""Drive the C ABI the way the Go cgo package does: its own
stream, device memory and copies — no torch — and compare with the oracle."""
import ctypes as C

import numpy as np
import pytest

from etcd_amd import _lib
from etcd_amd.quorum import batch
from tests import oracle_c as oc

pytestmark = pytest.mark.gpu


class Dev:
    def __init__(self):
        self.lib = _lib.load()
        self.ptrs = []

    def alloc(self, nbytes):
        p = C.c_void_p()
        _lib.check(self.lib.qb_malloc(nbytes, C.byref(p)), "qb_malloc")
        self.ptrs.append(p.value)
        return p.value

    def close(self):
        for p in self.ptrs:
            _lib.check(self.lib.qb_free(p), "qb_free")


def test_fixed_roundtrip_raw_abi():
    lib = _lib.load()
    _lib.check(lib.qb_set_device(0), "qb_set_device")
    st = C.c_void_p()
    _lib.check(lib.qb_stream_create(C.byref(st)), "qb_stream_create")
    d = Dev()
    n, G = 5, 100003
    match, vd, gr, _ = oc.gen_fixed(0x5EED0002, n, G)
    dm, dvd, dgr = d.alloc(match.nbytes), d.alloc(G), d.alloc(G)
    dc, dv = d.alloc(8 * G), d.alloc(G)
    for dst, src in ((dm, match), (dvd, vd), (dgr, gr)):
        _lib.check(lib.qb_copy_h2d_async(dst, src.ctypes.data, src.nbytes, st), "h2d")
    _lib.check(lib.qb_memset_async(dc, 0, 8 * G, st), "memset")
    _lib.check(lib.qb_dev_fixed_committed_vote(n, G, dm, dvd, dgr, dc, dv, st), "eval")
    c = np.empty(G, np.uint64)
    v = np.empty(G, np.uint8)
    _lib.check(lib.qb_copy_d2h_async(c.ctypes.data, dc, c.nbytes, st), "d2h")
    _lib.check(lib.qb_copy_d2h_async(v.ctypes.data, dv, v.nbytes, st), "d2h")
    _lib.check(lib.qb_stream_sync(st), "sync")
    ec, ev = oc.fixed_eval(n, match, vd, gr)
    assert np.array_equal(c, ec) and np.array_equal(v, ev)
    d.close()
    _lib.check(lib.qb_stream_destroy(st), "qb_stream_destroy")


def test_malloc_reports_enomem():
    lib = _lib.load()
    p = C.c_void_p()
    rc = lib.qb_malloc(1 << 50, C.byref(p))  # 1 PiB
    assert rc in (_lib.QB_ENOMEM, _lib.QB_EHIP)
    assert lib.qb_last_error()


class Stream:
    """qb_stream_create / sync / destroy plus a Dev allocator, as the cgo
    package holds them."""

    def __init__(self):
        self.lib = _lib.load()
        _lib.check(self.lib.qb_set_device(0), "qb_set_device")
        self.st = C.c_void_p()
        _lib.check(self.lib.qb_stream_create(C.byref(self.st)), "qb_stream_create")
        self.d = Dev()

    def up(self, a):
        a = np.ascontiguousarray(a)
        p = self.d.alloc(max(a.nbytes, 16))
        if a.nbytes:
            _lib.check(self.lib.qb_copy_h2d_async(p, a.ctypes.data, a.nbytes, self.st), "h2d")
        self.sync()   # the host array may be a temporary
        return p

    def zeros(self, nbytes, value=0):
        p = self.d.alloc(max(nbytes, 16))
        _lib.check(self.lib.qb_memset_async(p, value, max(nbytes, 16), self.st), "memset")
        return p

    def down(self, p, like):
        out = np.empty_like(like)
        _lib.check(self.lib.qb_copy_d2h_async(out.ctypes.data, p, out.nbytes, self.st), "d2h")
        self.sync()
        return out

    def sync(self):
        _lib.check(self.lib.qb_stream_sync(self.st), "sync")

    def close(self):
        self.sync()
        self.d.close()
        _lib.check(self.lib.qb_stream_destroy(self.st), "qb_stream_destroy")


def test_csr_committed_vote_raw_abi():
    """qb_host_compile_configs -> qb_dev_csr_committed_vote with the optional
    validation (qb_dev_csr_validate), no torch."""
    s = Stream()
    lib = s.lib
    G = 50000
    off, m, cfg, votes = oc.gen_csr(0x5EED0004, "joint", G)
    d_off, d_m, d_cfg, d_votes = s.up(off), s.up(m), s.up(cfg), s.up(votes)
    d_c, d_v, d_bad = s.zeros(8 * G), s.zeros(G), s.zeros(8)
    _lib.check(lib.qb_dev_csr_validate(G, 10, d_off, d_bad, s.st), "validate")
    _lib.check(lib.qb_dev_csr_committed_vote(G, 10, d_off, d_m, d_cfg, d_votes, d_c, d_v, s.st),
               "csr")
    c = s.down(d_c, np.empty(G, np.uint64))
    v = s.down(d_v, np.empty(G, np.uint8))
    assert s.down(d_bad, np.empty(1, np.uint64))[0] == 0
    ec, ev = oc.csr_eval(off, m, cfg, votes)
    assert np.array_equal(c, ec) and np.array_equal(v, ev)
    s.close()


def _seq_state(n, G):
    match, _, _, ts = oc.gen_fixed(0x5EED0005, n, G)
    st = {"match": match, "active": np.zeros(G, np.uint16), "term": np.full(G, 7, np.uint64),
          "term_start": ts, "last_index": match[0].copy(), "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    oc.commit_all(n, st["match"], ts, st["committed"])
    return st


def _records(rng, G, M, last, slots, higher=0.002):
    group = rng.integers(0, G, size=M).astype(np.uint32)
    flags = slots(group).astype(np.uint8)
    index = last[group] - rng.integers(0, 64, size=M).astype(np.uint64)
    u = rng.random(M)
    term = np.where(u < 0.01, 6, np.where(u < 0.01 + higher, 8, 7)).astype(np.uint64)
    return group, flags, index, term


@pytest.mark.parametrize("fused", [True, False, "split"])
def test_fixed_tracker_raw_abi(fused):
    """qb_dev_fixed_tracker_step (fused), qb_dev_fixed_tracker_bucket +
    qb_dev_fixed_tracker_apply (split) and qb_dev_fixed_apply_appresp +
    qb_dev_fixed_commit_advance (two calls) through the raw ABI vs the
    sequential oracle; stepdown_at follows each entry point's contract."""
    s = Stream()
    lib = s.lib
    n, G, M = 5, 60000, 90000
    rng = np.random.default_rng(3)
    st = _seq_state(n, G)
    d_match, d_term = s.up(st["match"]), s.up(st["term"])
    d_ts, d_cm = s.up(st["term_start"]), s.up(st["committed"])
    d_act = s.zeros(2 * (G + 1))
    d_sd = s.zeros(4 * G, 0xFF if fused else 0x11)   # the two-call form self-initialises
    d_adv, d_stats = s.zeros(G), s.zeros(64)
    group, flags, index, term = _records(rng, G, M, st["last_index"],
                                         lambda g: rng.integers(1, n, size=g.size))
    d_g, d_f, d_i, d_t = s.up(group), s.up(flags), s.up(index), s.up(term)
    stats = oc.appresp_sequential(n, G, (group, flags, index, term), st)
    if fused == "split":
        need = lib.qb_fixed_tracker_workspace_bytes(n, G, M)
        ws = s.zeros(need)
        _lib.check(lib.qb_dev_fixed_tracker_bucket(n, G, M, d_g, d_f, d_i, d_t, ws, need, s.st),
                   "bucket")
        _lib.check(lib.qb_dev_fixed_tracker_apply(n, G, M, d_g, d_f, d_i, d_t, d_term, d_ts,
                                                  d_match, None, d_act, d_cm, d_sd, d_adv, d_stats,
                                                  ws, need, s.st), "apply")
    elif fused:
        need = lib.qb_fixed_tracker_workspace_bytes(n, G, M)
        ws = s.zeros(need)
        _lib.check(lib.qb_dev_fixed_tracker_step(n, G, M, d_g, d_f, d_i, d_t, d_term, d_ts,
                                                 d_match, None, d_act, d_cm, d_sd, d_adv, d_stats,
                                                 ws, need, s.st), "step")
    else:
        _lib.check(lib.qb_dev_fixed_apply_appresp(n, G, M, d_g, d_f, d_i, d_t, d_term, d_match,
                                                  None, d_act, d_sd, d_stats, s.st), "apply")
        _lib.check(lib.qb_dev_fixed_commit_advance(n, G, d_match, d_ts, d_cm, d_adv, s.st),
                   "commit")
    assert np.array_equal(s.down(d_match, st["match"]), st["match"])
    assert np.array_equal(s.down(d_cm, st["committed"]), st["committed"])
    assert np.array_equal(s.down(d_act, np.empty(G, np.uint16)), st["active"])
    sd = s.down(d_sd, np.empty(G, np.uint32))
    assert np.array_equal(sd != 0xFFFFFFFF, st["stepped_down"].astype(bool))
    got = s.down(d_stats, np.empty(8, np.uint64))
    assert np.array_equal(got[:7], stats[:7])
    s.close()


def test_csr_tracker_raw_abi():
    """qb_dev_csr_tracker_step over compiled ragged configs with learners."""
    s = Stream()
    lib = s.lib
    G, M = 40000, 60000
    rng = np.random.default_rng(4)
    off, m, cfg, _ = oc.gen_csr(0x5EED0003, "ragged", G)
    sizes = np.diff(off.astype(np.int64))
    last = np.maximum.reduceat(m, off[:-1].astype(np.int64))
    st = {"match": m.copy(), "active": np.zeros(G, np.uint16),
          "term": np.full(G, 7, np.uint64), "term_start": last - np.uint64(10),
          "last_index": last, "committed": np.zeros(G, np.uint64),
          "stepped_down": np.zeros(G, np.uint8)}
    oc.csr_commit_all(off, cfg, st["match"], st["term_start"], st["committed"])
    d_off, d_cfg, d_match = s.up(off), s.up(cfg), s.up(st["match"])
    d_term, d_ts, d_cm = s.up(st["term"]), s.up(st["term_start"]), s.up(st["committed"])
    d_act, d_sd, d_stats = s.zeros(2 * (G + 1)), s.zeros(4 * G, 0xFF), s.zeros(64)
    group, flags, index, term = _records(
        rng, G, M, last, lambda g: rng.integers(0, 1 << 30, size=g.size) % sizes[g])
    d_g, d_f, d_i, d_t = s.up(group), s.up(flags), s.up(index), s.up(term)
    stats = oc.csr_appresp_sequential(off, cfg, (group, flags, index, term), st)
    need = lib.qb_csr_tracker_workspace_bytes(G, 11, M)
    ws = s.zeros(need)
    _lib.check(lib.qb_dev_csr_tracker_step(G, 11, d_off, d_cfg, M, d_g, d_f, d_i, d_t, d_term,
                                           d_ts, d_match, None, d_act, d_cm, d_sd, None, d_stats,
                                           ws, need, s.st), "csr step")
    assert np.array_equal(s.down(d_match, st["match"]), st["match"])
    assert np.array_equal(s.down(d_cm, st["committed"]), st["committed"])
    sd = s.down(d_sd, np.empty(G, np.uint32))
    assert np.array_equal(sd != 0xFFFFFFFF, st["stepped_down"].astype(bool))
    assert np.array_equal(s.down(d_stats, np.empty(8, np.uint64))[:7], stats[:7])
    s.close()


def test_votes_raw_abi():
    """qb_dev_record_votes + qb_dev_csr_tally_votes through the raw ABI against
    the sequential candidate oracle (tests/test_gpu_votes.py restatement)."""
    from tests.test_gpu_votes import sequential_votes
    s = Stream()
    lib = s.lib
    G, M = 3000, 9000
    rng = np.random.default_rng(5)
    cc = batch.compile_configs([set(rng.choice(20, size=int(rng.integers(1, 8)), replace=False)
                                    + 1) for _ in range(G)])
    gterm = rng.integers(5, 9, size=G).astype(np.uint64)
    group = rng.integers(0, G, size=M).astype(np.uint32)
    sizes = np.diff(cc.off.astype(np.int64))
    slot = (rng.integers(0, 1 << 20, size=M) % sizes[group]).astype(np.uint8)
    rej = rng.random(M) < 0.3
    flags = (slot | (rej.astype(np.uint8) << 7)).astype(np.uint8)
    u = rng.random(M)
    term = np.where(u < 0.05, gterm[group] - 1, np.where(u < 0.07, gterm[group] + 1,
                                                         gterm[group])).astype(np.uint64)
    want_votes, want_sd, want_dec, want_stats = sequential_votes(
        0, cc.cfg, np.zeros(G, np.uint32), gterm, group, flags, term)
    d_cfg, d_gt = s.up(cc.cfg), s.up(gterm)
    d_votes, d_sd, d_dec, d_stats = s.zeros(4 * G), s.zeros(4 * G), s.zeros(4 * G), s.zeros(64)
    d_g, d_f, d_t = s.up(group), s.up(flags), s.up(term)
    need = lib.qb_votes_workspace_bytes(M)
    ws = s.zeros(need)
    _lib.check(lib.qb_dev_record_votes(0, G, M, d_g, d_f, d_t, d_gt, d_cfg, d_votes, d_sd, d_dec,
                                       d_stats, ws, need, s.st), "record votes")
    res = s.zeros(G)
    _lib.check(lib.qb_dev_csr_tally_votes(G, d_cfg, d_votes, None, None, res, s.st), "tally")
    assert np.array_equal(s.down(d_votes, np.empty(G, np.uint32)), want_votes)
    assert np.array_equal(s.down(d_sd, np.empty(G, np.uint32)), want_sd)
    assert np.array_equal(s.down(d_dec, np.empty(G, np.uint32)), want_dec)
    assert np.array_equal(s.down(d_stats, np.empty(8, np.uint64)), want_stats)
    s.close()


def test_comm_allgather_world1_raw_abi():
    """The RCCL all-gather entry points on a single-rank communicator: unique
    ID -> init -> qb_dev_allgather_results (the node-wide vectors equal the
    shard) -> destroy."""
    s = Stream()
    lib = s.lib
    uid = (C.c_char * 128)()
    _lib.check(lib.qb_comm_get_unique_id(uid), "unique id")
    comm = C.c_void_p()
    _lib.check(lib.qb_comm_init(C.byref(comm), 1, 0, uid), "comm init")
    G = 100001
    c = np.arange(G, dtype=np.uint64) * np.uint64(3)
    v = (np.arange(G) % 3 + 1).astype(np.uint8)
    d_c, d_v = s.up(c), s.up(v)
    o_c, o_v = s.zeros(8 * G), s.zeros(G)
    need = lib.qb_allgather_workspace_bytes(G, 1)
    ws = s.zeros(need)
    _lib.check(lib.qb_dev_allgather_results(comm, G, d_c, d_v, o_c, o_v, ws, need, s.st),
               "allgather")
    assert np.array_equal(s.down(o_c, c), c) and np.array_equal(s.down(o_v, v), v)
    _lib.check(lib.qb_comm_destroy(comm), "comm destroy")
    s.close()


@pytest.mark.parametrize("n,frac,base", [(1, 1.0, 0), (4095, 0.5, 7), (1 << 20, 0.01, 123),
                                          (1000003, 1.0, 0), (5000, 0.0, 9)])
def test_compact_and_scatter_changed_raw_abi(n, frac, base):
    """qb_dev_compact_changed: the changed groups in group order as (g_base +
    g, commit) pairs and the device count; qb_dev_scatter_changed applies them
    (padding gid UINT32_MAX skipped)."""
    s = Stream()
    lib = s.lib
    rng = np.random.default_rng(n)
    changed = (rng.random(n) < frac).astype(np.uint8) * rng.integers(1, 256, n).astype(np.uint8)
    commit = rng.integers(0, 1 << 63, n, dtype=np.int64).astype(np.uint64) | np.uint64(1 << 63)
    d_ch, d_c = s.up(changed), s.up(commit)
    gid, val, cnt = s.zeros(4 * n + 8), s.zeros(8 * n + 8), s.zeros(8)
    need = lib.qb_compact_changed_workspace_bytes(n)
    ws = s.zeros(need)
    _lib.check(lib.qb_dev_compact_changed(n, d_ch, d_c, base, gid, val, cnt, ws, need, s.st),
               "compact")
    idx = np.nonzero(changed)[0]
    k = int(s.down(cnt, np.empty(1, np.uint64))[0])
    assert k == idx.size
    assert np.array_equal(s.down(gid, np.empty(n + 2, np.uint32))[:k], (idx + base).astype(np.uint32))
    assert np.array_equal(s.down(val, np.empty(n + 1, np.uint64))[:k], commit[idx])
    total = n + base
    out = s.up(np.zeros(total, np.uint64))
    pad = s.up(np.full(3, 0xFFFFFFFF, np.uint32))
    _lib.check(lib.qb_dev_scatter_changed(k, gid, val, total, out, s.st), "scatter")
    _lib.check(lib.qb_dev_scatter_changed(3, pad, val, total, out, s.st), "scatter padding")
    want = np.zeros(total, np.uint64)
    want[idx + base] = commit[idx]
    assert np.array_equal(s.down(out, np.empty(total, np.uint64)), want)
    s.close()


def test_allgather_changed_world1_raw_abi():
    """qb_dev_allgather_changed on a single-rank communicator over three ticks:
    commit_all carries every changed group's commit, *changed_total counts
    them, a tick with nothing changed moves nothing."""
    s = Stream()
    lib = s.lib
    uid = (C.c_char * 128)()
    _lib.check(lib.qb_comm_get_unique_id(uid), "unique id")
    comm = C.c_void_p()
    _lib.check(lib.qb_comm_init(C.byref(comm), 1, 0, uid), "comm init")
    G = 300007
    need = lib.qb_allgather_changed_workspace_bytes(G, 1)
    ws = s.zeros(need)
    d_all = s.up(np.zeros(G, np.uint64))
    want = np.zeros(G, np.uint64)
    rng = np.random.default_rng(5)
    for frac in (0.2, 0.0, 1.0):
        changed = (rng.random(G) < frac).astype(np.uint8)
        commit = rng.integers(0, 1 << 62, G, dtype=np.int64).astype(np.uint64)
        d_ch, d_c = s.up(changed), s.up(commit)
        n = C.c_uint64(99)
        _lib.check(lib.qb_dev_allgather_changed(comm, G, d_ch, d_c, d_all, C.byref(n), ws, need,
                                                s.st), "allgather changed")
        want = np.where(changed != 0, commit, want)
        assert n.value == int(changed.sum())
        assert np.array_equal(s.down(d_all, np.empty(G, np.uint64)), want)
    _lib.check(lib.qb_comm_destroy(comm), "comm destroy")
    s.close()


def _route_ref(total, world, grp, cols):
    """Stable partition by owner (shard_range) with rebased groups: the order
    etcd_amd/shard.py:route_records defines."""
    from etcd_amd.shard import shard_range
    bounds = np.array([shard_range(total, world, r)[1] for r in range(world)], np.int64)
    begins = np.array([shard_range(total, world, r)[0] for r in range(world)], np.int64)
    g = grp.astype(np.int64)
    owner = np.minimum(np.searchsorted(bounds, g, side="right"), world - 1)
    order = np.argsort(owner, kind="stable")
    out = {k: v[order] for k, v in cols.items()}
    out["group"] = (g - begins[owner])[order].astype(np.uint32)
    return out, np.bincount(owner, minlength=world)


@pytest.mark.parametrize("world,total,M,opt", [(1, 1000, 5000, True), (2, 100003, 300001, False),
                                               (3, 7, 20000, True), (8, 1 << 20, 1 << 20, True),
                                               (64, 100000, 70001, False), (5, 0, 1000, True)])
def test_route_partition_raw_abi(world, total, M, opt):
    """qb_dev_route_partition against the stable host partition: owners from
    qb_shard_range, groups >= total to the last rank, the columns moved in
    (owner, original position) order; send_off per destination."""
    s = Stream()
    lib = s.lib
    rng = np.random.default_rng(world * 7919 + M)
    hi = max(total + total // 50, 1) + 3
    cols = {"group": rng.integers(0, hi, M).astype(np.uint32),
            "flags": rng.integers(0, 256, M).astype(np.uint8),
            "index": rng.integers(0, 1 << 62, M).astype(np.uint64),
            "term": rng.integers(0, 1 << 62, M).astype(np.uint64)}
    if opt:
        cols["hint"] = rng.integers(0, 1 << 62, M).astype(np.uint64)
        cols["log_term"] = rng.integers(0, 1 << 62, M).astype(np.uint64)
    names = ("group", "flags", "index", "term", "hint", "log_term")
    din = {k: s.up(v) for k, v in cols.items()}
    dout = {k: s.zeros(v.nbytes) for k, v in cols.items()}
    off = s.zeros(4 * (world + 1))
    need = lib.qb_route_partition_workspace_bytes(world, M)
    ws = s.zeros(need)
    _lib.check(lib.qb_dev_route_partition(total, world, M, *[din.get(n) for n in names],
                                          *[dout.get(n) for n in names], off, ws, need, s.st),
               "route partition")
    ref, counts = _route_ref(total, world, cols["group"], cols)
    for k, v in cols.items():
        assert np.array_equal(s.down(dout[k], v), ref[k]), k
    o = s.down(off, np.empty(world + 1, np.uint32))
    assert np.array_equal(np.diff(o.astype(np.int64)), counts) and o[0] == 0 and o[-1] == M
    s.close()


def test_route_records_world1_raw_abi():
    """qb_dev_route_records on a single-rank communicator: every record stays,
    groups rebased (rank 0 begins at 0), order kept; an output capacity below
    the receive count is refused (QB_EINVAL) before anything moves."""
    s = Stream()
    lib = s.lib
    uid = (C.c_char * 128)()
    _lib.check(lib.qb_comm_get_unique_id(uid), "unique id")
    comm = C.c_void_p()
    _lib.check(lib.qb_comm_init(C.byref(comm), 1, 0, uid), "comm init")
    M, total = 200003, 50000
    rng = np.random.default_rng(5)
    cols = {"group": rng.integers(0, total + 100, M).astype(np.uint32),
            "flags": rng.integers(0, 256, M).astype(np.uint8),
            "index": rng.integers(0, 1 << 62, M).astype(np.uint64),
            "term": rng.integers(0, 1 << 62, M).astype(np.uint64)}
    names = ("group", "flags", "index", "term")
    din = {k: s.up(v) for k, v in cols.items()}
    dout = {k: s.zeros(v.nbytes) for k, v in cols.items()}
    need = lib.qb_route_workspace_bytes(1, M)
    ws = s.zeros(need)
    cnt = C.c_uint64(0)
    rc = lib.qb_dev_route_records(comm, total, M, *[din[n] for n in names], None, None,
                                  *[dout[n] for n in names], None, None, M - 1, C.byref(cnt),
                                  ws, need, s.st)
    assert rc == _lib.QB_EINVAL and b"capacity" in lib.qb_last_error()
    _lib.check(lib.qb_dev_route_records(comm, total, M, *[din[n] for n in names], None, None,
                                        *[dout[n] for n in names], None, None, M, C.byref(cnt),
                                        ws, need, s.st), "route records")
    assert cnt.value == M
    for k, v in cols.items():
        assert np.array_equal(s.down(dout[k], v), v), k
    _lib.check(lib.qb_comm_destroy(comm), "comm destroy")
    s.close()


def test_fixed_batches_raw_abi():
    """qb_dev_fixed_committed_vote_batches: several batches of one shape in
    one call over two streams (batch i on stream i % 2), each bit-exact vs
    the oracle; a bad batch stops the call with its error."""
    lib = _lib.load()
    _lib.check(lib.qb_set_device(0), "qb_set_device")
    sts = [C.c_void_p(), C.c_void_p()]
    for s in sts:
        _lib.check(lib.qb_stream_create(C.byref(s)), "qb_stream_create")
    d = Dev()
    n, G, B = 7, 30001, 5

    class FB(C.Structure):
        _fields_ = [(f, C.c_void_p) for f in ("match", "voted", "granted", "commit_out",
                                               "vote_out")]
    host, tab = [], (FB * B)()
    for b in range(B):
        match, vd, gr, _ = oc.gen_fixed(0x5EED0002, n, G, g_begin=b * G)
        dm, dvd, dgr, dc, dv = (d.alloc(match.nbytes), d.alloc(G), d.alloc(G), d.alloc(8 * G),
                                d.alloc(G))
        for dst, src in ((dm, match), (dvd, vd), (dgr, gr)):
            _lib.check(lib.qb_copy_h2d_async(dst, src.ctypes.data, src.nbytes, sts[0]), "h2d")
        tab[b] = FB(dm, dvd, dgr, dc, dv)
        host.append((match, vd, gr, dc, dv))
    _lib.check(lib.qb_stream_sync(sts[0]), "sync")
    streams = (C.c_void_p * 2)(sts[0].value, sts[1].value)
    _lib.check(lib.qb_dev_fixed_committed_vote_batches(n, G, B, tab, streams, 2), "batches")
    for s in sts:
        _lib.check(lib.qb_stream_sync(s), "sync")
    for match, vd, gr, dc, dv in host:
        c, v = np.empty(G, np.uint64), np.empty(G, np.uint8)
        _lib.check(lib.qb_copy_d2h_async(c.ctypes.data, dc, c.nbytes, sts[0]), "d2h")
        _lib.check(lib.qb_copy_d2h_async(v.ctypes.data, dv, v.nbytes, sts[0]), "d2h")
        _lib.check(lib.qb_stream_sync(sts[0]), "sync")
        ec, ev = oc.fixed_eval(n, match, vd, gr)
        assert np.array_equal(c, ec) and np.array_equal(v, ev)
    tab[2] = FB(None, None, None, host[2][3], None)  # commit_out without match
    assert lib.qb_dev_fixed_committed_vote_batches(n, G, B, tab, streams, 2) == _lib.QB_EINVAL
    assert lib.qb_dev_fixed_committed_vote_batches(n, G, B, tab, None, 0) == _lib.QB_EINVAL
    for s in sts:
        _lib.check(lib.qb_stream_sync(s), "sync")
    d.close()
    for s in sts:
        _lib.check(lib.qb_stream_destroy(s), "qb_stream_destroy")
