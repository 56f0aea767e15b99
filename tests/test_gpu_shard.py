"""The N > 1 path with the HIP kernels in the loop: two gloo ranks (both on
cuda:0 — the box has one GPU) each evaluate their shard_range of the
counter-generated groups with the device kernels, then assemble the node-wide
result (etcd_amd.shard.allgather_results) or deliver a record batch to the
owning shard (route_records) before the device tracker step; rank 0 compares
with the single-process C oracle over all groups, bit for bit.  gloo moves
host tensors, so the collectives run on the .cpu() copies (the driver's
multi-GPU bench runs the same calls over RCCL)."""
import os
import queue
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from etcd_amd.shard import shard_range

pytestmark = pytest.mark.gpu
SEED = 0x5EED0003


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args):
    """Run target on world ranks; rank 0's queued result.  A rank that dies
    before queueing fails the test at once (not after the queue timeout)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    deadline = time.monotonic() + 240
    while True:
        try:
            out = q.get(timeout=1)
            break
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead:
                for p in procs:
                    p.kill()
                pytest.fail(f"a rank exited with {dead[0]} before reporting")
            if time.monotonic() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail("no result within 240 s")
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    return out


def _eval_worker(rank, world, port, q, total, kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.quorum import batch
        from etcd_amd.shard import allgather_results
        dev = torch.device("cuda", 0)
        b, e = shard_range(total, world, rank)
        if kind == "fixed":
            grp = batch.FixedGroups.synth(SEED, 5, e - b, g_begin=b, device=dev)
        else:
            grp = batch.CsrGroups.synth(SEED, kind, e - b, g_begin=b, device=dev)
        c, v = grp.committed_vote()
        gc, gv = allgather_results(c.cpu(), v.cpu(), total)
        if rank == 0:
            q.put((gc.numpy().view(np.uint64).copy(), gv.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,total,kind", [(2, 100003, "fixed"), (2, 50001, "ragged"),
                                              (3, 30000, "joint")])
def test_sharded_device_eval_allgather(world, total, kind):
    from tests import oracle_c as oc
    gc, gv = _spawn(_eval_worker, world, total, kind)
    if kind == "fixed":
        match, vd, gr, _ = oc.gen_fixed(SEED, 5, total)
        ec, ev = oc.fixed_eval(5, match, vd, gr)
    else:
        off, m, cfg, votes = oc.gen_csr(SEED, kind, total)
        ec, ev = oc.csr_eval(off, m, cfg, votes)
    assert np.array_equal(gc, ec) and np.array_equal(gv, ev)


def _batch_of(rank, total, M, last):
    """Records arriving at ``rank``: global group numbers over every shard."""
    rng = np.random.default_rng(500 + rank)
    grp = rng.integers(0, total, M).astype(np.uint32)
    slot = rng.integers(1, 5, M).astype(np.uint8)
    idx = last[grp] - rng.integers(0, 64, M).astype(np.uint64)
    term = np.where(rng.random(M) < 0.02, 6, np.where(rng.random(M) < 0.002, 8, 7))
    return grp, slot, idx, term.astype(np.uint64)


def _tracker_worker(rank, world, port, q, total, M):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etcd_amd.quorum import batch
        from etcd_amd.shard import allgather_results, route_records
        from tests import oracle_c as oc
        dev = torch.device("cuda", 0)
        b, e = shard_range(total, world, rank)
        full, _, _, ts_full = oc.gen_fixed(SEED, 5, total)
        grp, slot, idx, term = _batch_of(rank, total, M, full[0])
        out = route_records({"group": torch.from_numpy(grp.view(np.int32)),
                             "flags": torch.from_numpy(slot),
                             "index": torch.from_numpy(idx.view(np.int64)),
                             "term": torch.from_numpy(term.view(np.int64))}, total)
        # this shard's leader state, regenerated from the counter-based spec
        match, _, _, ts = oc.gen_fixed(SEED, 5, e - b, g_begin=b)
        tr = batch.FixedTracker(5, e - b, dev)
        tr.match.copy_(batch.from_u64(match, dev))
        tr.term_start.copy_(batch.from_u64(ts, dev))
        tr.term.fill_(7)
        tr.commit_advance()
        tr.step(batch.AppRespBatch(out["group"].to(dev), out["flags"].to(dev),
                                   out["index"].to(dev), out["term"].to(dev)))
        rows = [allgather_results(tr.match[s].cpu(), tr.active[: e - b].to(torch.uint8).cpu(),
                                  total)[0] for s in range(5)]
        cm, sd = allgather_results(tr.committed.cpu(),
                                   tr.stepped_down().to(torch.uint8).cpu(), total)
        if rank == 0:
            q.put((np.stack([r.numpy().view(np.uint64) for r in rows]).copy(),
                   cm.numpy().view(np.uint64).copy(), sd.numpy().astype(bool)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_routed_records_device_tracker_step(world):
    """Batches arriving at every rank are routed to the owning shards
    (route_records, stable in (source rank, position) order) and applied by
    the bucketed device step there; the node-wide state equals the
    sequential oracle over the concatenated batches on all groups."""
    from tests import oracle_c as oc
    total, M = 60001, 50000
    match, cm, sd = _spawn(_tracker_worker, world, total, M)
    full, _, _, ts = oc.gen_fixed(SEED, 5, total)
    st = {"match": full.copy(), "active": np.zeros(total, np.uint16),
          "term": np.full(total, 7, np.uint64), "term_start": ts,
          "committed": np.zeros(total, np.uint64), "stepped_down": np.zeros(total, np.uint8)}
    oc.commit_all(5, st["match"], ts, st["committed"])
    for r in range(world):   # the global batch order route_records preserves per group
        grp, slot, idx, term = _batch_of(r, total, M, full[0])
        oc.appresp_sequential(5, total, (grp, slot, idx, term), st)
    assert np.array_equal(match, st["match"])
    assert np.array_equal(cm, st["committed"])
    assert np.array_equal(sd, st["stepped_down"].astype(bool))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_route_partition_device_matches_host(world):
    """shard.route_records' device partition (qb_dev_route_partition) equals
    its host twin on the same columns: the RCCL path and the gloo tests send
    identical runs."""
    from etcd_amd.shard import _partition_host, route_partition
    total, M = 60001, 100000
    rng = np.random.default_rng(world)
    cols = {"group": torch.from_numpy(rng.integers(0, total + 10, M).astype(np.int32)),
            "flags": torch.from_numpy(rng.integers(0, 256, M).astype(np.uint8)),
            "index": torch.from_numpy(rng.integers(0, 1 << 62, M)),
            "term": torch.from_numpy(rng.integers(0, 1 << 62, M))}
    hs, hc = _partition_host(cols, total, world, 0)
    ds, dc = route_partition({k: v.cuda() for k, v in cols.items()}, total, world)
    assert hc == dc
    for k in cols:
        assert torch.equal(hs[k], ds[k].cpu()), k


def _nccl_world1_worker(rank, world, port, q, total):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from etcd_amd.quorum import batch
        from etcd_amd.shard import allgather_results
        dev = torch.device("cuda", 0)
        grp = batch.FixedGroups.synth(SEED, 5, total, device=dev)
        c, v = grp.committed_vote()
        gc, gv = allgather_results(c, v, total)   # RCCL, device tensors
        torch.cuda.synchronize()
        q.put((bool(torch.equal(gc, c)), bool(torch.equal(gv, v)), gc.is_cuda, gc.numel()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_allgather_results_rccl_world1():
    """allgather_results over RCCL (backend "nccl", device tensors) on a
    single-rank group — the call the driver's multi-GPU bench makes, here with
    the one GPU (RCCL refuses two ranks on one device)."""
    ok_c, ok_v, on_dev, n = _spawn(_nccl_world1_worker, 1, 50_000)
    assert ok_c and ok_v and on_dev and n == 50_000


def _rccl_comm_world1_worker(rank, world, port, q, total):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from etcd_amd.comm import RcclComm
        from etcd_amd.quorum import batch
        dev = torch.device("cuda", 0)
        comm = RcclComm.from_process_group(dev)
        grp = batch.FixedGroups.synth(SEED, 5, total, device=dev)
        c, v = grp.committed_vote()
        gc, gv = comm.allgather_results(c, v, total)      # qb_dev_allgather_results
        ok_c = bool(torch.equal(gc, c))
        M = 10_000
        gen = torch.Generator(device=dev)
        gen.manual_seed(3)
        cols = {"group": torch.randint(0, total + 5, (M,), generator=gen, device=dev),  # int64
                "flags": torch.randint(0, 5, (M,), generator=gen, device=dev).to(torch.uint8),
                "index": torch.arange(M, device=dev, dtype=torch.int64).flip(0),
                "term": torch.full((M,), 7, dtype=torch.int64, device=dev)}
        got = comm.route_records(cols, total)               # qb_dev_route_records
        torch.cuda.synchronize()
        same = all(torch.equal(got[k].to(torch.int64), (cols[k] & 0xFFFFFFFF if k == "group"
                                                         else cols[k]).to(torch.int64))
                   for k in cols)
        # qb_dev_allgather_changed: the changed groups' commits land in the
        # node-wide vector (gc, from the full all-gather above)
        changed = (torch.arange(total, device=dev) % 7 == 3).to(torch.uint8)
        newc = c + 1000
        n = comm.allgather_changed(changed, newc, total, gc)
        torch.cuda.synchronize()
        delta_ok = n == int(changed.sum()) and bool(torch.equal(gc, torch.where(changed.bool(), newc, c)))
        comm.close()
        q.put((ok_c, bool(torch.equal(gv, v)), same, delta_ok, comm.world))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_comm_c_abi_world1():
    """etcd_amd.comm.RcclComm — the C ABI's communicator, what bench.py's N > 1
    path times — on a single-rank group: unique id over torch.distributed,
    qb_comm_init, the all-gather, the record routing (every record stays,
    in order, an int64 group column converted) and the changed-commit delta
    gather against the inputs."""
    ok_c, ok_v, ok_r, ok_d, w = _spawn(_rccl_comm_world1_worker, 1, 50_000)
    assert ok_c and ok_v and ok_r and ok_d and w == 1
