"""The C ABI's multi-rank exchange code (etcd_amd/csrc/qb_comm.cpp) at world
2, 3 and 8, on the box's one GPU: each rank is a host thread with its own HIP
stream, and the RCCL entry points qb_comm.cpp calls come from the test-only
tests/fake_rccl/fake_rccl.cpp (libqb_fakecomm.so = the product's objects +
that file instead of librccl; the product library is untouched).  RCCL
refuses two ranks on one GPU, so this is how the uneven-shard padding and
compaction of qb_dev_allgather_results, the count exchange / padded gathers /
full-gather fallback of qb_dev_allgather_changed, and the send/recv offsets of
qb_dev_route_records run before the driver's 8-GPU node — against the
single-process numpy restatement of the same rules (etcd_amd/shard.py
shard_range, the stable owner partition), including local failures on one
rank that every rank must report together (no rank left waiting).

Reference boundary replaced: server/etcdserver/api/rafthttp/peer.go:178 (the
per-group message delivery between members)."""
import ctypes as C
import os
import threading

import numpy as np
import pytest
import torch

from etcd_amd import _lib
from etcd_amd.shard import shard_range

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "tests", "fake_rccl", "libqb_fakecomm.so")
DEV = "cuda"
QB_EINVAL = -1

_fake = None


def fake():
    global _fake
    if _fake is None:
        if not os.path.exists(FAKE):
            raise RuntimeError(f"{FAKE} not built (make -C tests/fake_rccl, or "
                               "__graft_entry__.build())")
        lib = C.CDLL(FAKE)
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _fake = lib
    return _fake


def run_ranks(world, body, timeout=120):
    """body(rank, comm, stream) on `world` threads, each with its own
    communicator (qb_comm_init, collective) and stream; returns the results
    in rank order.  A thread still running after `timeout` fails the test
    (a rank left waiting in an exchange) instead of hanging the suite."""
    lib = fake()
    uid = C.create_string_buffer(128)
    assert lib.qb_comm_get_unique_id(uid) == 0
    out, errs = [None] * world, []

    def worker(r):
        try:
            assert lib.qb_set_device(0) == 0
            st = C.c_void_p()
            assert lib.qb_stream_create(C.byref(st)) == 0
            comm = C.c_void_p()
            rc = lib.qb_comm_init(C.byref(comm), world, r, uid)
            assert rc == 0, lib.qb_last_error()
            try:
                out[r] = body(r, comm, st)
                assert lib.qb_stream_sync(st) == 0
            finally:
                lib.qb_comm_destroy(comm)
                lib.qb_stream_destroy(st)
        except BaseException as ex:  # reported below
            errs.append((r, ex))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank is still waiting in an exchange"
    if errs:
        raise errs[0][1]
    return out


def _err():
    return fake().qb_last_error().decode()


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(DEV)


@pytest.mark.parametrize("world,total", [(2, 1 << 20), (3, 1000003), (8, 8 * 4099 + 5),
                                         (8, 7), (3, 0)])
def test_allgather_results_world_n(world, total):
    """qb_dev_allgather_results: every rank ends with the node-wide commit /
    vote vectors, shards in rank order — even shards gathered in place,
    uneven ones padded to the largest shard and compacted (total % world
    != 0), and shards of size 0 (total < world)."""
    rng = np.random.default_rng(world * 7 + total)
    commit = rng.integers(0, 1 << 63, size=total, dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, size=total).astype(np.uint64)   # full u64 range
    vote = rng.integers(0, 4, size=total).astype(np.uint8)
    d_commit, d_vote = u64(commit), torch.from_numpy(vote).to(DEV)
    lib = fake()
    ws_bytes = lib.qb_allgather_workspace_bytes(total, world)
    outs = [(torch.full((max(total, 1),), -1, dtype=torch.int64, device=DEV),
             torch.full((max(total, 1),), 0xEE, dtype=torch.uint8, device=DEV),
             torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=DEV)) for _ in range(world)]
    torch.cuda.synchronize()

    def body(r, comm, st):
        b, e = shard_range(total, world, r)
        ca, va, ws = outs[r]
        rc = lib.qb_dev_allgather_results(comm, total, d_commit[b:].data_ptr() if e > b else None,
                                          d_vote[b:].data_ptr() if e > b else None,
                                          ca.data_ptr(), va.data_ptr(), ws.data_ptr(), ws.numel(),
                                          st)
        assert rc == 0, _err()
    run_ranks(world, body)
    torch.cuda.synchronize()
    for r in range(world):
        ca, va, _ = outs[r]
        assert np.array_equal(ca[:total].cpu().numpy().view(np.uint64), commit), r
        assert np.array_equal(va[:total].cpu().numpy(), vote), r


def _delta_ticks(rng, total, world):
    """Changed sets of four ticks: 30 %, none, 1 %, every group, and one
    skewed tick (all of rank 0's shard, nothing elsewhere)."""
    b0, e0 = shard_range(total, world, 0)
    skew = np.zeros(total, bool)
    skew[b0:e0] = True
    return [rng.random(total) < 0.3, np.zeros(total, bool), rng.random(total) < 0.01,
            np.ones(total, bool), skew]


@pytest.mark.parametrize("world,total", [(2, 200000), (3, 100003), (8, 8 * 5001 + 3)])
def test_allgather_changed_world_n(world, total):
    """qb_dev_allgather_changed over five ticks: the node-wide commit vector
    every rank keeps equals the start vector with every changed group's new
    commit — through the padded (gid, commit) gathers for sparse ticks and
    the full-gather fallback for the dense and skewed ones (12 B x the
    largest count > 8 B x the shard cap)."""
    rng = np.random.default_rng(world * 11 + total)
    lib = fake()
    want = rng.integers(0, 1 << 62, size=total, dtype=np.uint64)
    ws_bytes = lib.qb_allgather_changed_workspace_bytes(total, world)
    alls = [u64(want) for _ in range(world)]
    wss = [torch.empty(ws_bytes, dtype=torch.uint8, device=DEV) for _ in range(world)]
    for tick, changed in enumerate(_delta_ticks(rng, total, world)):
        commit = want.copy()
        commit[changed] = rng.integers(0, 1 << 63, size=int(changed.sum()), dtype=np.uint64)
        d_commit = u64(commit)
        d_changed = torch.from_numpy(changed.astype(np.uint8)).to(DEV)
        torch.cuda.synchronize()

        def body(r, comm, st):
            b, e = shard_range(total, world, r)
            n = C.c_uint64(0)
            rc = lib.qb_dev_allgather_changed(comm, total, d_changed[b:].data_ptr(),
                                              d_commit[b:].data_ptr(), alls[r].data_ptr(),
                                              C.byref(n), wss[r].data_ptr(), wss[r].numel(), st)
            assert rc == 0, _err()
            return int(n.value)
        got_n = run_ranks(world, body)
        torch.cuda.synchronize()
        assert got_n == [int(changed.sum())] * world, tick
        want = commit
        for r in range(world):
            assert np.array_equal(alls[r].cpu().numpy().view(np.uint64), want), (tick, r)


def test_allgather_changed_local_failure_reaches_every_rank():
    """rank 1 passes a NULL changed column.  Its compaction fails,
    the failure travels as a ~0 count, and EVERY rank returns QB_EINVAL —
    none is left waiting in the count exchange or the pair gathers."""
    world, total = 3, 30001
    lib = fake()
    d_changed = torch.ones(total, dtype=torch.uint8, device=DEV)
    d_commit = torch.arange(total, dtype=torch.int64, device=DEV)
    ca = [torch.zeros(total, dtype=torch.int64, device=DEV) for _ in range(world)]
    ws_bytes = lib.qb_allgather_changed_workspace_bytes(total, world)
    wss = [torch.empty(ws_bytes, dtype=torch.uint8, device=DEV) for _ in range(world)]
    torch.cuda.synchronize()

    def body(r, comm, st):
        b, _ = shard_range(total, world, r)
        n = C.c_uint64(0)
        rc = lib.qb_dev_allgather_changed(comm, total,
                                          None if r == 1 else d_changed[b:].data_ptr(),
                                          d_commit[b:].data_ptr(), ca[r].data_ptr(), C.byref(n),
                                          wss[r].data_ptr(), wss[r].numel(), st)
        return rc, _err()
    res = run_ranks(world, body)
    assert all(rc == QB_EINVAL for rc, _ in res), res
    assert "NULL" in res[1][1]                              # the failing rank's own reason
    assert all("rank 1 failed" in msg for r, (_, msg) in enumerate(res) if r != 1), res


def _route_expected(batches, total, world):
    """Per destination rank: every source's records it owns, in (source rank,
    source position) order, group rebased to the owner's local index; a group
    >= total goes to the last rank (index >= its shard size)."""
    ends = np.array([shard_range(total, world, r)[1] for r in range(world)], np.int64)
    begins = np.array([shard_range(total, world, r)[0] for r in range(world)], np.int64)
    exp = [{k: [] for k in batches[0]} for _ in range(world)]
    for src in batches:
        g = src["group"].astype(np.int64)
        owner = np.minimum(np.searchsorted(ends, g, side="right"), world - 1)
        for d in range(world):
            sel = owner == d
            for k, col in src.items():
                exp[d][k].append((g[sel] - begins[d]).astype(np.uint32) if k == "group"
                                 else col[sel])
    return [{k: np.concatenate(v) for k, v in e.items()} for e in exp]


@pytest.mark.parametrize("world,total,with_hint", [(2, 1 << 20, True), (3, 100003, False),
                                                   (8, 8 * 3001 + 7, True)])
def test_route_records_world_n(world, total, with_hint):
    """qb_dev_route_records: ranks hold batches of different sizes (one of
    them empty) with groups anywhere in the node, a few past `total`; every
    rank receives exactly the records it owns, stably, with all columns."""
    rng = np.random.default_rng(world * 13 + total)
    lib = fake()
    sizes = [int(rng.integers(1000, 60000)) for _ in range(world)]
    sizes[1] = 0
    names = ("group", "flags", "index", "term") + (("hint", "log_term") if with_hint else ())
    host, dev = [], []
    for r in range(world):
        M = sizes[r]
        g = rng.integers(0, total, size=M).astype(np.uint32)
        g[rng.random(M) < 0.01] = np.uint32(total + 5)
        h = {"group": g, "flags": rng.integers(0, 256, size=M).astype(np.uint8),
             "index": rng.integers(0, 1 << 63, size=M, dtype=np.uint64),
             "term": rng.integers(0, 1 << 40, size=M, dtype=np.uint64)}
        if with_hint:
            h["hint"] = rng.integers(0, 1 << 63, size=M, dtype=np.uint64)
            h["log_term"] = rng.integers(0, 1 << 20, size=M, dtype=np.uint64)
        host.append(h)
        dev.append({k: (torch.from_numpy(v.view(np.int32) if k == "group" else
                                         v.view(np.int64) if v.dtype == np.uint64 else v)
                        .to(DEV) if M else torch.zeros(1, dtype=torch.int64, device=DEV))
                    for k, v in h.items()})
    exp = _route_expected(host, total, world)
    cap = sum(sizes)
    outs = [{k: torch.zeros(cap, dtype=torch.int64, device=DEV) for k in names}
            for _ in range(world)]
    wss = [torch.empty(lib.qb_route_workspace_bytes(world, sizes[r]) or 1, dtype=torch.uint8,
                       device=DEV) for r in range(world)]
    torch.cuda.synchronize()

    def body(r, comm, st):
        p = lambda d, k: d[k].data_ptr() if k in d and k in names else None  # noqa: E731
        cnt = C.c_uint64(0)
        rc = lib.qb_dev_route_records(comm, total, sizes[r],
                                      *[p(dev[r], k) for k in ("group", "flags", "index", "term",
                                                               "hint", "log_term")],
                                      *[p(outs[r], k) for k in ("group", "flags", "index", "term",
                                                                "hint", "log_term")],
                                      cap, C.byref(cnt), wss[r].data_ptr(), wss[r].numel(), st)
        assert rc == 0, _err()
        return int(cnt.value)
    counts = run_ranks(world, body)
    torch.cuda.synchronize()
    for d in range(world):
        n = counts[d]
        assert n == len(exp[d]["group"]), d
        for k in names:
            raw = outs[d][k].cpu().numpy().view(np.uint8)
            w = exp[d][k].dtype.itemsize
            got = raw[: n * w].view(exp[d][k].dtype)
            assert np.array_equal(got, exp[d][k]), (d, k)


@pytest.mark.parametrize("fail", ["capacity", "null_output"])
def test_route_records_local_failure_reaches_every_rank(fail):
    """One rank cannot take its records (out_cap too small, or a NULL output
    column, advertised as capacity 0): every rank returns QB_EINVAL with the
    same decision, and none is left in a send."""
    world, total, M = 3, 30000, 5000
    lib = fake()
    rng = np.random.default_rng(5)
    cols = [{"group": torch.from_numpy(rng.integers(0, total, size=M).astype(np.int32)).to(DEV),
             "flags": torch.zeros(M, dtype=torch.uint8, device=DEV),
             "index": torch.arange(M, dtype=torch.int64, device=DEV),
             "term": torch.ones(M, dtype=torch.int64, device=DEV)} for _ in range(world)]
    outs = [{k: torch.zeros(world * M, dtype=torch.int64, device=DEV)
             for k in ("group", "flags", "index", "term")} for _ in range(world)]
    wss = [torch.empty(lib.qb_route_workspace_bytes(world, M), dtype=torch.uint8, device=DEV)
           for _ in range(world)]
    torch.cuda.synchronize()

    def body(r, comm, st):
        cap = 10 if (fail == "capacity" and r == 2) else world * M
        o = dict(outs[r])
        if fail == "null_output" and r == 2:
            o["term"] = None
        p = lambda d, k: d[k].data_ptr() if d.get(k) is not None else None  # noqa: E731
        cnt = C.c_uint64(0)
        rc = lib.qb_dev_route_records(comm, total, M,
                                      *[p(cols[r], k) for k in ("group", "flags", "index", "term")],
                                      None, None,
                                      *[p(o, k) for k in ("group", "flags", "index", "term")],
                                      None, None, cap, C.byref(cnt), wss[r].data_ptr(),
                                      wss[r].numel(), st)
        return rc, _err()
    res = run_ranks(world, body)
    assert all(rc == QB_EINVAL for rc, _ in res), res
    assert all("rank 2 would receive" in msg for _, msg in res), res
