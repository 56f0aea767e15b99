"""The node-wide collectives through the C ABI's RCCL communicator — the
calls a Go embedder binds (include/quorum_batch.h: qb_comm_init,
qb_dev_allgather_results, qb_dev_route_records), not torch's collectives.

SURVEY.md §8e: groups shard by id over the GPUs of one node; RCCL over xGMI
is used only to all-gather the per-shard commit/vote vectors into the
node-wide result, and to deliver record batches that arrive at any rank to
the rank owning their group.  The communicator's unique id travels over the
embedder's own channel; here that channel is torch.distributed's default
process group (one broadcast of 128 bytes at construction).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch
import torch.distributed as dist

from etcd_amd import _lib

QB_COMM_ID_BYTES = 128
_ROUTE_COLS = ("group", "flags", "index", "term", "hint", "log_term")


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


class RcclComm:
    """One rank's qb_comm (RCCL communicator over the node's GPUs)."""

    def __init__(self, world: int, rank: int, device, uid: bytes):
        if len(uid) != QB_COMM_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        self.world, self.rank, self.device = world, rank, torch.device(device)
        self._uid = C.create_string_buffer(uid, QB_COMM_ID_BYTES)
        self._h = C.c_void_p()
        _lib.call("qb_comm_init", C.byref(self._h), world, rank, self._uid)
        self._ws = None

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(QB_COMM_ID_BYTES)
        _lib.call("qb_comm_get_unique_id", buf)
        return buf.raw

    @classmethod
    def from_process_group(cls, device, group: Optional[dist.ProcessGroup] = None) -> "RcclComm":
        """Rank 0 makes the id; torch.distributed carries it to every rank."""
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        return cls(world, rank, device, box[0])

    def close(self) -> None:
        if self._h:
            _lib.call("qb_comm_destroy", self._h)
            self._h = C.c_void_p()

    def _shard_len(self, total: int) -> int:
        from etcd_amd.shard import shard_range
        b, e = shard_range(total, self.world, self.rank)
        return e - b

    @staticmethod
    def _check_device(name: str, t: torch.Tensor) -> None:
        if t.device.type != "cuda":
            raise ValueError(f"{name}: a device tensor is required (got {t.device})")

    def _check(self, name: str, t: torch.Tensor, numel: int, sizes) -> None:
        """The C side reads ``numel`` elements from the raw device pointer: a
        wrong length, a host tensor or another element size would be an
        out-of-bounds device read (or a fault inside RCCL), so refuse it."""
        self._check_device(name, t)
        if t.element_size() not in sizes:
            raise ValueError(f"{name}: element size {t.element_size()}, expected {sizes}")
        if t.numel() != numel:
            raise ValueError(f"{name}: {t.numel()} elements, expected {numel}")
        if not t.is_contiguous():
            raise ValueError(f"{name}: must be contiguous")

    def _pg_ok(self) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() == self.world

    def _agree(self, err: Optional[str], extra=None, agree: bool = True):
        """Decide the callers' argument checks on every rank together (ADVICE
        r4): a refusal on one rank alone would leave the others waiting in the
        RCCL exchange.  When torch.distributed spans the same ranks, one
        all-reduce (SUM) carries [failed, *extra]; every rank raises if any
        rank refused.  Returns the summed ``extra`` (or None).  Without a
        process group the embedder's own channel must agree (the C ABI's
        route exchange decides its own failures collectively).

        ``agree=False``: no all-reduce and no host sync — the
        local checks still run and raise on this rank.  For a per-tick caller
        whose arguments keep the shapes an earlier agreed call accepted on
        every rank (the same tensors, the same ``total``); the exchange then
        costs only itself."""
        if not agree or not self._pg_ok():
            if err:
                raise ValueError(err)
            return None
        vals = [1 if err else 0] + list(extra or [])
        dev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor(vals, dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        if int(t[0].item()):
            raise ValueError(err or f"{int(t[0].item())} other rank(s) refused their arguments")
        return [int(x) for x in t[1:].tolist()]

    def _checked(self, checks) -> Optional[str]:
        """Run the argument checks locally; the first refusal's text."""
        try:
            for c in checks:
                c()
        except ValueError as ex:
            return str(ex)
        return None

    def _workspace(self, nbytes: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.device)
        return self._ws

    def allgather_results(self, commit: torch.Tensor, vote: torch.Tensor, total: int,
                          commit_all: Optional[torch.Tensor] = None,
                          vote_all: Optional[torch.Tensor] = None, agree: bool = True):
        """Node-wide commit (u64) / vote (u8) vectors from this rank's shard
        (qb_dev_allgather_results; shard_range order).  ``commit`` / ``vote``
        hold exactly this rank's shard_range (device, 8-byte / 1-byte).
        Every rank passes the same ``total``; a refused argument on any rank
        raises ValueError on every rank (``_agree``; ``agree=False``: see
        there)."""
        n = self._shard_len(total)
        if commit_all is None:
            commit_all = torch.empty(total, dtype=torch.int64, device=self.device)
        if vote_all is None:
            vote_all = torch.empty(total, dtype=torch.uint8, device=self.device)
        self._agree(self._checked([lambda: self._check("commit", commit, n, (8,)),
                                   lambda: self._check("vote", vote, n, (1,)),
                                   lambda: self._check("commit_all", commit_all, total, (8,)),
                                   lambda: self._check("vote_all", vote_all, total, (1,))]),
                    agree=agree)
        need = _lib.fn("qb_allgather_workspace_bytes")(total, self.world)
        ws = self._workspace(need)
        _lib.call("qb_dev_allgather_results", self._h, total, commit.data_ptr(), vote.data_ptr(),
                  commit_all.data_ptr(), vote_all.data_ptr(), ws.data_ptr(), ws.numel(),
                  _stream(self.device))
        return commit_all, vote_all

    def allgather_changed(self, changed: torch.Tensor, commit: torch.Tensor, total: int,
                          commit_all: torch.Tensor, agree: bool = True) -> int:
        """Apply every rank's changed-commit delta (qb_dev_allgather_changed)
        to ``commit_all`` (device, total u64 kept across ticks, updated in
        place).  ``changed`` (u8) / ``commit``: this rank's shard.  Returns the
        number of changed groups node-wide.  Every rank passes the same
        ``total``; a refused argument on any rank raises on every rank
        (``agree=False``: see ``_agree``)."""
        n = self._shard_len(total)
        err = None
        if changed.dtype not in (torch.uint8, torch.bool):
            err = "allgather_changed: changed must be uint8 / bool"
        else:
            changed = changed.contiguous().view(torch.uint8)
            commit = commit.contiguous()
            err = self._checked([lambda: self._check("changed", changed, n, (1,)),
                                 lambda: self._check("commit", commit, n, (8,)),
                                 lambda: self._check("commit_all", commit_all, total, (8,))])
        self._agree(err, agree=agree)
        need = _lib.fn("qb_allgather_changed_workspace_bytes")(total, self.world)
        ws = self._workspace(need)
        n = C.c_uint64(0)
        _lib.call("qb_dev_allgather_changed", self._h, total, changed.data_ptr(), commit.data_ptr(),
                  commit_all.data_ptr(), C.byref(n), ws.data_ptr(), ws.numel(),
                  _stream(self.device))
        return int(n.value)

    def route_records(self, cols: Dict[str, torch.Tensor], total: int,
                      out_cap: Optional[int] = None,
                      agree: bool = True) -> Dict[str, torch.Tensor]:
        """This rank's records after delivery (qb_dev_route_records): every
        rank's records for groups of this shard, group rebased to the local
        index, in (source rank, source position) order.  ``out_cap`` must
        bound the records this rank receives; by default it is the sum of
        every rank's batch size (all-reduced over torch.distributed when it is
        initialised — ranks may hold batches of different sizes — else world x
        this rank's M).  Ranks may pass different ``out_cap`` values, or some
        none: the all-reduce runs on every rank either way, and it also
        carries the column checks, so a rank whose columns are refused raises
        together with every other rank (the C ABI then decides capacity
        overflows collectively itself).  ``agree=False`` (see ``_agree``)
        needs ``out_cap``: without the all-reduce no rank knows the others'
        batch sizes."""
        from etcd_amd.shard import _device_columns
        if not agree and out_cap is None:
            raise ValueError("route_records: agree=False needs out_cap")
        err, M = None, 0
        try:
            cols = _device_columns(cols)
            for name, col in cols.items():
                self._check_device(f"route_records: column {name!r}", col)
            M = cols["group"].numel()
        except ValueError as ex:
            err = str(ex)
        summed = self._agree(err, [M], agree=agree)
        if out_cap is None:
            out_cap = summed[0] if summed is not None else self.world * M
        out = {}
        for name, col in cols.items():
            out[name] = torch.empty(max(out_cap, 1), dtype=col.dtype, device=self.device)
        need = _lib.fn("qb_route_workspace_bytes")(self.world, M)
        ws = self._workspace(need)
        count = C.c_uint64(0)

        def p(d, n):
            t = d.get(n)
            return t.data_ptr() if t is not None else None
        _lib.call("qb_dev_route_records", self._h, total, M, *[p(cols, n) for n in _ROUTE_COLS],
                  *[p(out, n) for n in _ROUTE_COLS], out_cap, C.byref(count), ws.data_ptr(),
                  ws.numel(), _stream(self.device))
        return {n: t[: count.value] for n, t in out.items()}
