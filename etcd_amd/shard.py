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
    backend = dist.get_backend(group)
    if backend == "nccl" and total == cap * world:
        # equal shards (the bench's weak-scaling case): gathered straight into
        # the node-wide vectors, no padding copies and no concatenation
        gc = torch.empty(total, dtype=commit.dtype, device=commit.device)
        gv = torch.empty(total, dtype=vote.dtype, device=vote.device)
        dist.all_gather_into_tensor(gc, commit.contiguous(), group=group)
        dist.all_gather_into_tensor(gv, vote.contiguous(), group=group)
        return gc, gv
    pc = torch.zeros(cap, dtype=commit.dtype, device=commit.device)
    pv = torch.zeros(cap, dtype=vote.dtype, device=vote.device)
    pc[: e - b] = commit
    pv[: e - b] = vote
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
    dev = cols["group"].device
    if dev.type == "cuda":  # the device partition (HIP, qb_route.hip), groups rebased
        send, sc = route_partition(cols, total, world)
    else:                   # host tensors (gloo tests): the same partition in torch
        send, sc = _partition_host(cols, total, world, dist.get_rank(group))
    send_counts = torch.tensor(sc, dtype=torch.int64, device=dev)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rc = recv_counts.tolist()
    out = {}
    for name, col in send.items():
        recv = torch.empty((sum(rc),) + tuple(col.shape[1:]), dtype=col.dtype, device=dev)
        dist.all_to_all_single(recv, col, output_split_sizes=rc, input_split_sizes=sc,
                               group=group)
        out[name] = recv
    return out


def _owner_host(g: torch.Tensor, total: int, world: int) -> torch.Tensor:
    bounds = torch.tensor([shard_range(total, world, r)[1] for r in range(world)],
                          dtype=torch.int64, device=g.device)
    return torch.bucketize(g, bounds, right=True).clamp_(max=world - 1)


def _partition_host(cols, total, world, rank):
    g = cols["group"].to(torch.int64) & 0xFFFFFFFF
    owner = _owner_host(g, total, world)
    order = torch.argsort(owner, stable=True)
    begins = torch.tensor([shard_range(total, world, r)[0] for r in range(world)],
                          dtype=torch.int64, device=g.device)
    send = {name: col[order].contiguous() for name, col in cols.items()}
    send["group"] = (g - begins[owner])[order].to(torch.int32)
    return send, torch.bincount(owner, minlength=world).tolist()


_ROUTE_COLS = ("group", "flags", "index", "term", "hint", "log_term")
_WIDE = (torch.int64, torch.uint64) if hasattr(torch, "uint64") else (torch.int64,)
_INTS = (torch.int8, torch.uint8, torch.int16, torch.int32, torch.int64) + _WIDE[1:]


def _device_columns(cols: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """The column layout qb_dev_route_partition reads, whatever the caller
    passed — as the host path accepts: group as int32 (any integer dtype,
    masked to uint32 like the host path), flags uint8, the 8-byte columns
    int64/uint64, every column contiguous and of one length.  An unsupported
    dtype raises ValueError instead of being read as the wrong bytes."""
    for need in ("group", "flags", "index", "term"):
        if need not in cols:
            raise ValueError(f"route_partition: column {need!r} is required")
    M = cols["group"].numel()
    out = {}
    for name, col in cols.items():
        if col.device != cols["group"].device:
            raise ValueError(f"route_partition: column {name!r} is on {col.device}, group on "
                             f"{cols['group'].device}")
        if col.dim() != 1 or col.numel() != M:
            raise ValueError(f"route_partition: column {name!r} must be 1-D of length {M}")
        if name == "group":
            if col.dtype not in _INTS:
                raise ValueError(f"route_partition: group must be an integer tensor, not {col.dtype}")
            if col.dtype != torch.int32:
                col = (col.to(torch.int64) & 0xFFFFFFFF).to(torch.int32)  # wraps: uint32 bits
        elif name == "flags":
            if col.dtype not in (torch.uint8, torch.int8):
                raise ValueError(f"route_partition: flags must be uint8, not {col.dtype}")
            col = col.view(torch.uint8)
        elif col.dtype not in _WIDE:
            raise ValueError(f"route_partition: {name} must be int64/uint64, not {col.dtype}")
        out[name] = col.contiguous()
    return out


def route_partition(cols: Dict[str, torch.Tensor], total: int, world: int):
    """The device half of the routing (qb_dev_route_partition): ``cols``
    (device; group, flags, index, term required, hint / log_term optional)
    stably partitioned by owner rank, group rebased to the owner's local
    index.  Returns (send columns, per-rank counts)."""
    from etcd_amd import _lib
    lib = _lib.load()
    unknown = set(cols) - set(_ROUTE_COLS)
    if unknown:
        raise ValueError(f"route_partition: unknown columns {sorted(unknown)}")
    cols = _device_columns(cols)
    dev = cols["group"].device
    M = cols["group"].numel()
    send = {name: torch.empty_like(col) for name, col in cols.items()}
    off = torch.empty(world + 1, dtype=torch.int32, device=dev)
    nbytes = lib.qb_route_partition_workspace_bytes(world, M)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)

    def ptr(d, name):
        t = d.get(name)
        return t.data_ptr() if t is not None else None
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.qb_dev_route_partition(
        total, world, M, *[ptr(cols, n) for n in _ROUTE_COLS], *[ptr(send, n) for n in _ROUTE_COLS],
        off.data_ptr(), ws.data_ptr(), nbytes, stream), "qb_dev_route_partition")
    o = off.cpu().tolist()
    return send, [o[r + 1] - o[r] for r in range(world)]


def compact_changed(changed: torch.Tensor, commit: torch.Tensor, g_base: int = 0):
    """The changed-commit delta of a shard: (global group u32 as int32, new
    commit) of the groups whose ``changed`` flag (u8) is set, in group order —
    a group surfaces a Ready when its commit moved (raft/node.go:573,
    raft/rawnode.go:157).  Device tensors run qb_dev_compact_changed (HIP);
    host tensors the same compaction in torch."""
    if changed.numel() != commit.numel():
        raise ValueError("changed and commit differ in length")
    if changed.device != commit.device:
        raise ValueError(f"changed is on {changed.device}, commit on {commit.device}")
    if changed.dtype not in (torch.uint8, torch.bool):
        raise ValueError(f"changed must be uint8/bool, not {changed.dtype}")
    if commit.dtype not in _WIDE:
        raise ValueError(f"commit must be int64/uint64, not {commit.dtype}")
    if g_base + commit.numel() > 0xFFFFFFFF:
        raise ValueError("global groups must fit uint32")
    changed = changed.contiguous().view(torch.uint8)
    commit = commit.contiguous()
    if commit.device.type != "cuda":
        idx = torch.nonzero(changed, as_tuple=True)[0]
        return (idx + g_base).to(torch.int32), commit[idx]
    from etcd_amd import _lib
    lib = _lib.load()
    n = commit.numel()
    dev = commit.device
    gid = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(n, 1), dtype=commit.dtype, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    nbytes = lib.qb_compact_changed_workspace_bytes(n)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    _lib.check(lib.qb_dev_compact_changed(n, changed.data_ptr(), commit.data_ptr(), g_base,
                                          gid.data_ptr(), val.data_ptr(), cnt.data_ptr(),
                                          ws.data_ptr(), nbytes,
                                          torch.cuda.current_stream(dev).cuda_stream),
               "qb_dev_compact_changed")
    k = int(cnt.item())
    return gid[:k], val[:k]


def allgather_changed(changed: torch.Tensor, commit: torch.Tensor, total: int,
                      commit_all: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> int:
    """Apply every rank's changed-commit delta to ``commit_all`` (the
    node-wide vector the caller keeps across ticks; updated in place) — 12
    bytes per changed group exchanged instead of allgather_results' whole
    vectors.  ``changed`` / ``commit``: this rank's shard.
    Returns the number of changed groups node-wide.  One count exchange, then
    one padded all-gather per column (padding gid = -1, i.e. UINT32_MAX)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    b, e = shard_range(total, world, rank)
    if commit.numel() != e - b or changed.numel() != e - b:
        raise ValueError("local vectors do not match this rank's shard")
    if commit_all.numel() != total:
        raise ValueError("commit_all must hold every group")
    gid, val = compact_changed(changed, commit, b)
    dev = commit.device
    n = torch.tensor([gid.numel()], dtype=torch.int64, device=dev)
    counts = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    if mx == 0:
        return 0
    pg = torch.full((mx,), -1, dtype=torch.int32, device=dev)
    pv = torch.zeros(mx, dtype=val.dtype, device=dev)
    pg[: gid.numel()] = gid
    pv[: val.numel()] = val
    lg = [torch.empty_like(pg) for _ in range(world)]
    lv = [torch.empty_like(pv) for _ in range(world)]
    dist.all_gather(lg, pg, group=group)
    dist.all_gather(lv, pv, group=group)
    g_all, v_all = torch.cat(lg), torch.cat(lv)
    keep = g_all != -1
    idx = g_all[keep].to(torch.int64) & 0xFFFFFFFF
    commit_all[idx] = v_all[keep].to(commit_all.dtype)
    return sum(counts)
