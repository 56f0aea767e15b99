"""N > 1 path on CPU: world_size 2 (and 3) gloo processes each evaluate their
shard of the counter-generated groups and all-gather the node-wide result.

No GPU exists here, so each rank's shard is evaluated by the C oracle as a
stand-in for the kernel; what is under test is the sharding (ranges, global
group numbering, independent regeneration per shard) and the gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from etcd_amd.shard import shard_range

SEED = 0x5EED0003


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.shard import allgather_results
        from tests import oracle_c as oc
        b, e = shard_range(total, world, rank)
        if kind == "fixed":
            match, vd, gr, _ = oc.gen_fixed(SEED, 5, e - b, g_begin=b)
            c, v = oc.fixed_eval(5, match, vd, gr)
        else:
            off, m, cfg, votes = oc.gen_csr(SEED, kind, e - b, g_begin=b)
            c, v = oc.csr_eval(off, m, cfg, votes)
        gc, gv = allgather_results(torch.from_numpy(c.view(np.int64)), torch.from_numpy(v), total)
        if rank == 0:
            q.put((gc.numpy().view(np.uint64).copy(), gv.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_shard_range_partition():
    for total in (0, 1, 7, 100, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1 and sizes[0] == max(sizes)


@pytest.mark.parametrize("world,total,kind", [(2, 10001, "fixed"), (2, 4096, "ragged"),
                                              (3, 5000, "joint")])
def test_sharded_eval_allgather_equals_single_process(world, total, kind):
    from tests import oracle_c as oc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, kind, q))
             for r in range(world)]
    for p in procs:
        p.start()
    gc, gv = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if kind == "fixed":
        match, vd, gr, _ = oc.gen_fixed(SEED, 5, total)
        ec, ev = oc.fixed_eval(5, match, vd, gr)
    else:
        off, m, cfg, votes = oc.gen_csr(SEED, kind, total)
        ec, ev = oc.csr_eval(off, m, cfg, votes)
    assert np.array_equal(gc, ec) and np.array_equal(gv, ev)


def _route_inputs(rank, M, total):
    rng = np.random.default_rng(1000 + rank)
    grp = rng.integers(0, total + 3, M).astype(np.uint32)  # a few past the end
    idx = rng.integers(0, 1 << 40, M).astype(np.uint64)
    flags = rng.integers(0, 256, M).astype(np.uint8)
    return grp, idx, flags


def _route_worker(rank, world, port, total, M, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.shard import route_records
        grp, idx, flags = _route_inputs(rank, M, total)
        out = route_records({"group": torch.from_numpy(grp.view(np.int32)),
                             "index": torch.from_numpy(idx.view(np.int64)),
                             "flags": torch.from_numpy(flags)}, total)
        q.put((rank, out["group"].numpy().view(np.uint32).copy(),
               out["index"].numpy().view(np.uint64).copy(), out["flags"].numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_route_records_by_owning_shard(world):
    total, M = 1000, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_route_worker, args=(r, world, port, total, M, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (g, i, f)) for r, g, i, f in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    inputs = [_route_inputs(r, M, total) for r in range(world)]
    for r in range(world):
        b, e = shard_range(total, world, r)
        last = r == world - 1
        want_g, want_i, want_f = [], [], []
        for src in range(world):  # (source rank, source position) order
            g, i, f = inputs[src]
            sel = ((g >= b) & (g < e)) | ((g >= total) & last)
            want_g.append(g[sel] - b)
            want_i.append(i[sel])
            want_f.append(f[sel])
        assert np.array_equal(got[r][0], np.concatenate(want_g).astype(np.uint32))
        assert np.array_equal(got[r][1], np.concatenate(want_i))
        assert np.array_equal(got[r][2], np.concatenate(want_f))


def _delta_inputs(total, tick, frac):
    """A tick's node-wide changed flags and new commits (the same on every
    rank: each takes its shard)."""
    rng = np.random.default_rng(77 + tick)
    changed = (rng.random(total) < frac).astype(np.uint8)
    commit = rng.integers(0, 1 << 63, total, dtype=np.int64).astype(np.uint64)
    commit[:3] = [0, (1 << 64) - 1, 1 << 63]  # the full u64 range travels
    return changed, commit


def _delta_worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.shard import allgather_changed
        b, e = shard_range(total, world, rank)
        commit_all = torch.zeros(total, dtype=torch.int64)
        seen = []
        for tick, frac in enumerate((0.3, 0.0, 0.01, 1.0)):
            changed, commit = _delta_inputs(total, tick, frac)
            n = allgather_changed(torch.from_numpy(changed[b:e]),
                                  torch.from_numpy(commit[b:e].view(np.int64)), total, commit_all)
            seen.append((n, commit_all.numpy().view(np.uint64).copy()))
        q.put((rank, seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 1001), (3, 5000)])
def test_allgather_changed_keeps_node_wide_commits(world, total):
    """shard.allgather_changed over gloo: after every tick each rank's
    node-wide vector equals applying every changed group's new commit (ticks
    with 30 %, 0 %, 1 % and 100 % of the groups changed, uneven shards)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_delta_worker, args=(r, world, port, total, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.zeros(total, np.uint64)
    for tick, frac in enumerate((0.3, 0.0, 0.01, 1.0)):
        changed, commit = _delta_inputs(total, tick, frac)
        want = np.where(changed != 0, commit, want)
        for r in range(world):
            n, vec = got[r][tick]
            assert n == int(changed.sum())
            assert np.array_equal(vec, want)


def test_compact_changed_host():
    from etcd_amd.shard import compact_changed
    changed, commit = _delta_inputs(777, 0, 0.2)
    gid, val = compact_changed(torch.from_numpy(changed), torch.from_numpy(commit.view(np.int64)), 40)
    idx = np.nonzero(changed)[0]
    assert np.array_equal(gid.numpy().astype(np.int64), idx + 40)
    assert np.array_equal(val.numpy().view(np.uint64), commit[idx])


def _comm_agree_worker(rank, world, port, q):
    """RcclComm's argument checks decided on every rank together:
    the object is built without qb_comm_init (no RCCL here); the checks run
    before any C call, so a refusal on one rank must raise on all ranks
    instead of leaving the others in the exchange."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.comm import RcclComm
        c = RcclComm.__new__(RcclComm)
        c.world, c.rank, c.device = world, rank, torch.device("cpu")
        c._check_device = lambda name, t: None   # host tensors stand in for device ones here
        res = []
        # only rank 1's column is refused (a host tensor, and an int32 term)
        M = 8 + rank
        cols = {"group": torch.zeros(M, dtype=torch.int32), "flags": torch.zeros(M, dtype=torch.uint8),
                "index": torch.zeros(M, dtype=torch.int64),
                "term": torch.zeros(M, dtype=torch.int32 if rank == 1 else torch.int64)}
        try:
            c.route_records(cols, 100)
            res.append("no error")
        except ValueError as ex:
            res.append(str(ex))
        except Exception as ex:  # e.g. the C call: must not be reached
            res.append(f"other {type(ex).__name__}")
        # agreement with extras: every rank's M summed, no refusal
        res.append(c._agree(None, [M]))
        # a refusal on rank 0 only, through allgather_results' checks
        try:
            c.allgather_results(torch.zeros(3 if rank == 0 else 50, dtype=torch.int64),
                                torch.zeros(50, dtype=torch.uint8), 100)
            res.append("no error")
        except ValueError as ex:
            res.append(str(ex))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_rccl_comm_argument_refusals_raise_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_comm_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    r0, r1 = got[0], got[1]
    assert "term" in r1[0] and "refused" in r0[0]      # rank 1's refusal raised on rank 0 too
    assert r0[1] == r1[1] == [8 + 9]
    assert "commit" in r0[2] and "refused" in r1[2]
