"""Sharding of raft groups over the GPUs of one node.

Groups are independent, so a shard is a contiguous range of global group
numbers evaluated by one rank with no data exchange.  The two collectives are
at the edges of the path: assembling the node-wide result (an all-gather of
the per-shard commit u64 and vote u8 vectors) and, for record batches that
arrive at arbitrary ranks, delivering each record to its group's shard (an
all-to-all) — RCCL (backend "nccl") on the GPU path, any torch.distributed
backend in tests.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[begin, end) of the groups owned by ``rank``: contiguous, sizes differ by
    at most one group."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def allgather_results(commit: torch.Tensor, vote: torch.Tensor, total: int,
                      group: Optional[dist.ProcessGroup] = None):
    """Node-wide commit/vote vectors from per-shard ones (shard_range order).

    Shards are padded to the largest shard so one all-gather per vector
    suffices; the padding is dropped afterwards."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    b, e = shard_range(total, world, rank)
    if commit.numel() != e - b or vote.numel() != e - b:
        raise ValueError("local vectors do not match this rank's shard")
    cap = shard_range(total, world, 0)[1]  # rank 0 holds the largest shard
    pc = torch.zeros(cap, dtype=commit.dtype, device=commit.device)
    pv = torch.zeros(cap, dtype=vote.dtype, device=vote.device)
    pc[: e - b] = commit
    pv[: e - b] = vote
    backend = dist.get_backend(group)
    if backend == "nccl":
        gc = torch.empty(world * cap, dtype=commit.dtype, device=commit.device)
        gv = torch.empty(world * cap, dtype=vote.dtype, device=vote.device)
        dist.all_gather_into_tensor(gc, pc, group=group)
        dist.all_gather_into_tensor(gv, pv, group=group)
        gc, gv = gc.view(world, cap), gv.view(world, cap)
    else:
        lc = [torch.empty_like(pc) for _ in range(world)]
        lv = [torch.empty_like(pv) for _ in range(world)]
        dist.all_gather(lc, pc, group=group)
        dist.all_gather(lv, pv, group=group)
        gc, gv = torch.stack(lc), torch.stack(lv)
    parts_c, parts_v = [], []
    for r in range(world):
        rb, re_ = shard_range(total, world, r)
        parts_c.append(gc[r, : re_ - rb])
        parts_v.append(gv[r, : re_ - rb])
    return torch.cat(parts_c), torch.cat(parts_v)


def route_records(cols: Dict[str, torch.Tensor], total: int,
                  group: Optional[dist.ProcessGroup] = None) -> Dict[str, torch.Tensor]:
    """Deliver every rank's records to the rank owning their group (SURVEY.md
    §8e: message batches are bucketed by owning shard).

    ``cols`` holds equal-length record columns, one of them ``"group"`` with
    global group numbers (int32 holding uint32).  Returns this rank's records
    with ``group`` rebased to the shard (local index), in (source rank,
    source position) order — a fixed batch order, which is what the leader
    step's sequential semantics need.  A group number >= total goes to the
    last rank as an out-of-range local index (counted there as a bad group).
    One count exchange plus one all-to-all per column: RCCL over xGMI on the
    GPU path, any torch.distributed backend in tests."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = cols["group"].device
    g = cols["group"].to(torch.int64) & 0xFFFFFFFF
    bounds = torch.tensor([shard_range(total, world, r)[1] for r in range(world)],
                          dtype=torch.int64, device=dev)
    owner = torch.bucketize(g, bounds, right=True).clamp_(max=world - 1)
    order = torch.argsort(owner, stable=True)
    send_counts = torch.bincount(owner, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    out = {}
    for name, col in cols.items():
        send = col[order].contiguous()
        recv = torch.empty((sum(rc),) + tuple(col.shape[1:]), dtype=col.dtype, device=dev)
        dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc,
                               group=group)
        out[name] = recv
    b, _ = shard_range(total, world, rank)
    local = (out["group"].to(torch.int64) & 0xFFFFFFFF) - b
    out["group"] = local.to(torch.int32)
    return out
