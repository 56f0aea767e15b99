"""Capacity: the node-wide sizes of BASELINE configs[3] (64M joint groups)
and configs[4] (128M groups) on ONE device, and the exchange code at the
index widths the 8-GPU run addresses (node-wide vectors of 2^27 entries).
Each bit-exact against the C oracle on the whole range or on sampled ranges,
or against an independent device restatement of the same rule (the routing's
stable owner partition, the delta scatter) over the whole range.

Reference call sites: raft/quorum/joint.go:49-75 (configs[3]),
raft/raft.go:1106-1259 with tracker/progress.go:144-153 (configs[4]),
server/etcdserver/api/rafthttp/peer.go:178 (the per-group delivery the
routing and gathers replace)."""
import ctypes as C

import numpy as np
import pytest
import torch

from etcd_amd import _lib
from etcd_amd.quorum import batch
from etcd_amd.shard import shard_range
from tests import oracle_c as oc
from tests import parity_checks as pc

pytestmark = pytest.mark.gpu
DEV = "cuda"
T27 = 1 << 27


@pytest.mark.timeout(600)
def test_csr_joint_64m_groups_one_device():
    """configs[3]'s whole node (64M JointConfig 5+5 groups, ~480M slots: CSR
    offsets near 2^29) in one k_csr launch: the full range equals eight
    independently synthesised and evaluated 8M-group pieces (small indexes),
    and three 1M-group windows (start, the 2^25 boundary, end) equal the C
    oracle."""
    seed, G, P = 0x5EED0004, 1 << 26, 1 << 23
    grp = batch.CsrGroups.synth(seed, "joint", G, device=DEV)
    assert int(grp.off[-1].item()) > (1 << 28)
    c = torch.empty(G, dtype=torch.int64, device=DEV)
    v = torch.empty(G, dtype=torch.uint8, device=DEV)
    grp.committed_vote(c, v)
    torch.cuda.synchronize()
    del grp
    torch.cuda.empty_cache()
    for o in range(0, G, P):
        piece = batch.CsrGroups.synth(seed, "joint", P, g_begin=o, device=DEV)
        pcm, pvt = piece.committed_vote()
        assert torch.equal(c[o:o + P], pcm) and torch.equal(v[o:o + P], pvt), o
        del piece, pcm, pvt
    threads = pc.host_threads()
    W = 1 << 20
    for w0 in (0, (1 << 25) - W // 2, G - W):
        off, m, cfg, votes = oc.gen_csr(seed, "joint", W, w0)
        ec, ev = oc.csr_eval(off, m, cfg, votes, threads=threads)
        assert np.array_equal(batch.as_u64(c[w0:w0 + W]), ec), w0
        assert np.array_equal(v[w0:w0 + W].cpu().numpy(), ev), w0


@pytest.mark.timeout(600)
def test_fixed_tracker_tick_128m_groups_one_device():
    """configs[4]'s whole node (128M 5-voter groups, 128M MsgAppResp records,
    2048 super-buckets) in one qb_dev_fixed_tracker_step on one device: the
    bench's stream tick against the sequential C oracle over every group
    (match, committed, active, stepdown) and every stat counter."""
    pc.check_tracker_stream(torch.device(DEV), False, T27, 1)


def _owner(g, total, world):
    ends = torch.tensor([shard_range(total, world, r)[1] for r in range(world)], dtype=torch.int64,
                        device=g.device)
    return torch.bucketize(g, ends, right=True).clamp_(max=world - 1)


@pytest.mark.timeout(600)
def test_route_partition_2e27():
    """qb_dev_route_partition at total = M = 2^27 over 8 owners (the node-wide
    record batch of configs[4]): the send offsets are the owner counts and
    each owner's run holds exactly its records in source order (the index
    column carries the source position) with the group rebased — checked on
    the device over the whole batch."""
    world, M = 8, T27
    g = torch.randint(0, T27, (M,), dtype=torch.int64, device=DEV)
    g[::997] = T27 + 3                                   # past the node: the last rank
    cols = {"group": g.to(torch.int32), "flags": torch.randint(0, 256, (M,), dtype=torch.uint8,
                                                                 device=DEV),
            "index": torch.arange(M, dtype=torch.int64, device=DEV),
            "term": torch.randint(0, 1 << 40, (M,), dtype=torch.int64, device=DEV)}
    out = {k: torch.empty_like(t) for k, t in cols.items()}
    send_off = torch.empty(world + 1, dtype=torch.int32, device=DEV)
    ws = torch.empty(_lib.fn("qb_route_partition_workspace_bytes")(world, M), dtype=torch.uint8,
                     device=DEV)
    _lib.call("qb_dev_route_partition", T27, world, M, cols["group"].data_ptr(),
              cols["flags"].data_ptr(), cols["index"].data_ptr(), cols["term"].data_ptr(), None, None,
              out["group"].data_ptr(), out["flags"].data_ptr(), out["index"].data_ptr(),
              out["term"].data_ptr(), None, None, send_off.data_ptr(), ws.data_ptr(), ws.numel(),
              torch.cuda.current_stream().cuda_stream)
    owner = _owner(g, T27, world)
    counts = torch.bincount(owner, minlength=world)
    want_off = torch.zeros(world + 1, dtype=torch.int64, device=DEV)
    want_off[1:] = torch.cumsum(counts, 0)
    assert torch.equal(send_off.long(), want_off)
    order = torch.argsort(owner, stable=True)
    assert torch.equal(out["index"], order)               # stable, by owner
    begins = torch.tensor([shard_range(T27, world, r)[0] for r in range(world)], dtype=torch.int64,
                          device=DEV)
    assert torch.equal(out["group"].long() & 0xFFFFFFFF, (g - begins[owner])[order])
    assert torch.equal(out["flags"], cols["flags"][order])
    assert torch.equal(out["term"], cols["term"][order])


@pytest.mark.timeout(600)
def test_compact_and_scatter_changed_2e27():
    """The delta's device halves at node scale: qb_dev_compact_changed of the
    last of 8 shards (global ids near 2^27) and qb_dev_scatter_changed of
    2^27 (gid, commit) pairs — a permutation of the node, with padding —
    into a 2^27-entry node-wide vector, against torch on the device."""
    world = 8
    b, e = shard_range(T27, world, world - 1)
    n = e - b
    changed = (torch.rand(n, device=DEV) < 0.4).to(torch.uint8)
    commit = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=DEV)
    gid = torch.empty(n, dtype=torch.int32, device=DEV)
    val = torch.empty(n, dtype=torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    ws = torch.empty(_lib.fn("qb_compact_changed_workspace_bytes")(n), dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("qb_dev_compact_changed", n, changed.data_ptr(), commit.data_ptr(), b, gid.data_ptr(),
              val.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), st)
    sel = torch.nonzero(changed.bool()).flatten()
    k = int(cnt.item())
    assert k == sel.numel()
    assert torch.equal(gid[:k].long() & 0xFFFFFFFF, sel + b) and torch.equal(val[:k], commit[sel])
    # scatter: every node group once (a permutation) plus padding entries
    m = T27 + (1 << 20)
    perm = torch.randperm(T27, device=DEV)
    g_all = torch.full((m,), -1, dtype=torch.int32, device=DEV)   # UINT32_MAX: skipped
    pos = torch.randperm(m, device=DEV)[:T27]
    g_all[pos] = perm.to(torch.int32)
    v_all = torch.randint(-(1 << 62), 1 << 62, (m,), dtype=torch.int64, device=DEV)
    node = torch.full((T27,), 7, dtype=torch.int64, device=DEV)
    _lib.call("qb_dev_scatter_changed", m, g_all.data_ptr(), v_all.data_ptr(), T27, node.data_ptr(), st)
    want = torch.empty(T27, dtype=torch.int64, device=DEV)
    want[perm] = v_all[pos]
    assert torch.equal(node, want)


@pytest.mark.timeout(300)
def test_allgather_results_rccl_world1_2e27():
    """qb_dev_allgather_results through RCCL (world 1) at total = 2^27."""
    from etcd_amd.comm import RcclComm
    comm = RcclComm(1, 0, DEV, RcclComm.unique_id())
    try:
        c = torch.randint(-(1 << 62), 1 << 62, (T27,), dtype=torch.int64, device=DEV)
        v = torch.randint(0, 4, (T27,), dtype=torch.uint8, device=DEV)
        ca, va = comm.allgather_results(c, v, T27)
        torch.cuda.synchronize()
        assert torch.equal(ca, c) and torch.equal(va, v)
    finally:
        comm.close()


@pytest.mark.timeout(600)
def test_fake_comm_world8_node_sizes():
    """The C ABI's world-8 exchange code (tests/fake_rccl, 8 host threads on
    one GPU) at the driver's node-wide sizes: qb_dev_allgather_results and
    qb_dev_allgather_changed over total = 2^27 + 5 (uneven shards, so the
    padded path), and qb_dev_route_records with 2^24 records per rank over a
    2^27-group node."""
    from tests.test_gpu_comm_fake import fake, run_ranks
    lib = fake()
    world, total = 8, T27 + 5
    commit = torch.randint(-(1 << 62), 1 << 62, (total,), dtype=torch.int64, device=DEV)
    vote = torch.randint(0, 4, (total,), dtype=torch.uint8, device=DEV)
    ws_b = lib.qb_allgather_workspace_bytes(total, world)
    torch.cuda.synchronize()

    def gather(r, comm, st):
        b, _ = shard_range(total, world, r)
        ca = torch.empty(total, dtype=torch.int64, device=DEV)
        va = torch.empty(total, dtype=torch.uint8, device=DEV)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=DEV)
        rc = lib.qb_dev_allgather_results(comm, total, commit[b:].data_ptr(), vote[b:].data_ptr(),
                                          ca.data_ptr(), va.data_ptr(), ws.data_ptr(), ws.numel(), st)
        assert rc == 0, lib.qb_last_error()
        assert lib.qb_stream_sync(st) == 0
        return bool(torch.equal(ca, commit)) and bool(torch.equal(va, vote))
    assert run_ranks(world, gather, timeout=300) == [True] * world
    torch.cuda.empty_cache()
    # the delta: 30 % of the node changes; every rank's node-wide vector follows
    before = torch.randint(-(1 << 62), 1 << 62, (total,), dtype=torch.int64, device=DEV)
    changed = (torch.rand(total, device=DEV) < 0.3).to(torch.uint8)
    after = torch.where(changed.bool(), commit, before)
    dws_b = lib.qb_allgather_changed_workspace_bytes(total, world)
    torch.cuda.synchronize()

    def delta(r, comm, st):
        b, _ = shard_range(total, world, r)
        node = before.clone()
        ws = torch.empty(dws_b, dtype=torch.uint8, device=DEV)
        torch.cuda.synchronize()
        nn = C.c_uint64(0)
        rc = lib.qb_dev_allgather_changed(comm, total, changed[b:].data_ptr(), after[b:].data_ptr(),
                                          node.data_ptr(), C.byref(nn), ws.data_ptr(), ws.numel(), st)
        assert rc == 0, lib.qb_last_error()
        assert lib.qb_stream_sync(st) == 0
        return int(nn.value), bool(torch.equal(node, after))
    res = run_ranks(world, delta, timeout=300)
    assert res == [(int(changed.sum().item()), True)] * world
    torch.cuda.empty_cache()
    # routing: 2^24 records per rank, groups anywhere in the node
    M = 1 << 24
    recs = [{"group": torch.randint(0, total, (M,), dtype=torch.int64, device=DEV),
             "flags": torch.randint(0, 256, (M,), dtype=torch.uint8, device=DEV),
             "index": torch.arange(M, dtype=torch.int64, device=DEV) + r * M,
             "term": torch.full((M,), r, dtype=torch.int64, device=DEV)} for r in range(world)]
    for rr in recs:
        rr["g32"] = rr["group"].to(torch.int32)
    rws_b = lib.qb_route_workspace_bytes(world, M)
    torch.cuda.synchronize()

    def route(r, comm, st):
        cap = world * M // 4        # the expected share is M: room for skew
        out = {"group": torch.empty(cap, dtype=torch.int32, device=DEV),
               "flags": torch.empty(cap, dtype=torch.uint8, device=DEV),
               "index": torch.empty(cap, dtype=torch.int64, device=DEV),
               "term": torch.empty(cap, dtype=torch.int64, device=DEV)}
        ws = torch.empty(rws_b, dtype=torch.uint8, device=DEV)
        torch.cuda.synchronize()
        cnt = C.c_uint64(0)
        src = recs[r]
        rc = lib.qb_dev_route_records(comm, total, M, src["g32"].data_ptr(), src["flags"].data_ptr(),
                                      src["index"].data_ptr(), src["term"].data_ptr(), None, None,
                                      out["group"].data_ptr(), out["flags"].data_ptr(),
                                      out["index"].data_ptr(), out["term"].data_ptr(), None, None,
                                      cap, C.byref(cnt), ws.data_ptr(), ws.numel(), st)
        assert rc == 0, lib.qb_last_error()
        assert lib.qb_stream_sync(st) == 0
        k = int(cnt.value)
        b, _ = shard_range(total, world, r)
        want_idx = torch.cat([s["index"][_owner(s["group"], total, world) == r] for s in recs])
        want_g = torch.cat([s["group"][_owner(s["group"], total, world) == r] for s in recs]) - b
        return (k == want_idx.numel() and bool(torch.equal(out["index"][:k], want_idx))
                and bool(torch.equal(out["group"][:k].long(), want_g)))
    assert run_ranks(world, route, timeout=300) == [True] * world
