"""Wire ingest (include/quorum_batch.h ``qb_dev_ingest_messages``): raw
protobuf raftpb.Message bytes (raft/raftpb/raft.proto:68-86) decoded on the
device into leader-inbox records for ``LeaderGroups.step``.  Validation is
the generated gogoproto Message.Unmarshal (raftpb/raft.pb.go:1739-2061)."""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib
from ._checks import check_tensors as _check_tensors
from .leader import LeaderInbox

WIRE_OK, WIRE_UNMARSHAL, WIRE_TYPE, WIRE_CTX = 0, 1, 2, 3
REC_NO_PROGRESS = 0x40


def pack_messages(msgs, groups, device="cuda"):
    """Host helper: a list of encoded messages and their envelope groups ->
    (bytes u8, msg_off int64 [M+1], msg_group int32) device tensors."""
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs), np.uint8) if msgs else np.zeros(0, np.uint8)
    dev = torch.device(device)
    b = torch.from_numpy(buf.copy() if buf.size else np.zeros(1, np.uint8)).to(dev)
    return (b, int(off[-1]), torch.from_numpy(off.view(np.int64).copy()).to(dev),
            torch.from_numpy(np.asarray(groups, np.uint32).view(np.int32).copy()).to(dev))


def group_rows(off: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """The 64-byte group-row table of a CSR slot-ID config
    (qb_dev_wire_group_rows): build once per config, pass to ``ingest(rows=)``."""
    G = off.numel() - 1
    rows = torch.empty(max(G, 1) * 8, dtype=torch.int64, device=off.device)
    _lib.call("qb_dev_wire_group_rows", G, off.data_ptr(), ids.data_ptr(), rows.data_ptr(),
              torch.cuda.current_stream(off.device).cuda_stream)
    return rows


def _check_batch(buf, nbytes, msg_off, msg_group):
    """The message batch: nbytes >= 0 bytes of buf, M + 1 offsets, M groups."""
    if not isinstance(nbytes, int) or nbytes < 0:
        raise _lib.QuorumBatchError(f"nbytes must be a non-negative int, got {nbytes!r}")
    M = msg_group.numel() if isinstance(msg_group, torch.Tensor) else 0
    _check_tensors(((buf, "buf", (torch.uint8,), nbytes),
                    (msg_off, "msg_off", (torch.int64,), M + 1),
                    (msg_group, "msg_group", (torch.int32,), 0)))


def ingest(buf: torch.Tensor, nbytes: int, msg_off: torch.Tensor, msg_group: torch.Tensor,
           off: torch.Tensor, ids: torch.Tensor, stats: torch.Tensor = None,
           rows: torch.Tensor = None):
    """Decode M = len(msg_group) messages.  ``off`` [G+1] int32 and ``ids``
    [off[G]] int64 are the groups' CSR slot IDs (ascending per group); with
    ``rows`` (``group_rows(off, ids)``) each message gathers one 64-byte row
    instead (qb_dev_ingest_messages_rows).
    Returns (LeaderInbox, status u8 tensor, msg_type u8 tensor)."""
    _check_batch(buf, nbytes, msg_off, msg_group)
    _check_tensors(((off, "off", (torch.int32,), 1), (ids, "ids", (torch.int64,), 0),
                    (stats, "stats", (torch.int64,), 4)))
    dev = buf.device
    M = msg_group.numel()
    G = off.numel() - 1
    _check_tensors(((rows, "rows", (torch.int64,), 8 * G), (buf, "buf", (torch.uint8,), 0),
                    (off, "off", (torch.int32,), 0)))
    n = max(M, 1)
    rg = torch.empty(n, dtype=torch.int32, device=dev)
    rf = torch.empty(n, dtype=torch.uint8, device=dev)
    ri, rt, rh, rl = (torch.empty(n, dtype=torch.int64, device=dev) for _ in range(4))
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    mtype = torch.empty(n, dtype=torch.uint8, device=dev)
    if rows is None:
        _lib.call("qb_dev_ingest_messages", M, buf.data_ptr(), nbytes, msg_off.data_ptr(),
                  msg_group.data_ptr(), G, off.data_ptr(), ids.data_ptr(), rg.data_ptr(),
                  rf.data_ptr(), ri.data_ptr(), rt.data_ptr(), rh.data_ptr(), rl.data_ptr(),
                  status.data_ptr(), mtype.data_ptr(),
                  None if stats is None else stats.data_ptr(),
                  torch.cuda.current_stream(dev).cuda_stream)
    else:
        _lib.call("qb_dev_ingest_messages_rows", M, buf.data_ptr(), nbytes, msg_off.data_ptr(),
                  msg_group.data_ptr(), G, rows.data_ptr(), ids.data_ptr(), rg.data_ptr(),
                  rf.data_ptr(), ri.data_ptr(), rt.data_ptr(), rh.data_ptr(), rl.data_ptr(),
                  status.data_ptr(), mtype.data_ptr(),
                  None if stats is None else stats.data_ptr(),
                  torch.cuda.current_stream(dev).cuda_stream)
    ib = LeaderInbox(rg, rf, ri, rt, rh, rl)
    ib._m = M
    return ib, status[:M], mtype[:M]


def ingest_tracker_step(tracker, buf: torch.Tensor, nbytes: int, msg_off: torch.Tensor,
                        msg_group: torch.Tensor, rows: torch.Tensor = None,
                        off: torch.Tensor = None, ids: torch.Tensor = None,
                        advanced_out: torch.Tensor = None, wire_stats: torch.Tensor = None,
                        reset_stats: bool = True, rearm: bool = True) -> torch.Tensor:
    """The composed tick in one call: M encoded responses decoded and stepped
    into ``tracker``, the commit advanced — ``ingest`` followed by
    ``tracker.step`` on its records, without the record columns between them
    (a message that is not a MsgAppResp steps nothing).  A
    ``batch.FixedTracker`` (qb_dev_ingest_fixed_tracker_step: ``rows``
    (``group_rows``) or ``off`` + ``ids`` give the groups' slot IDs) or a
    ``batch.CsrTracker`` (qb_dev_ingest_csr_tracker_step: ``ids`` over the
    tracker's own ``off``, ``rows`` optional).  ``reset_stats`` / ``rearm``
    as the trackers' ``step``; ``wire_stats`` (int64 [4], nullable)
    accumulates the QB_WIRE_* counts.  Returns the per-message status (u8 [M])."""
    from .batch import CsrTracker
    _check_batch(buf, nbytes, msg_off, msg_group)
    G = tracker.G
    _check_tensors(((buf, "buf", (torch.uint8,), 0), (tracker.committed, "tracker", (torch.int64,), G),
                    (rows, "rows", (torch.int64,), 8 * G),
                    (off, "off", (torch.int32,), G + 1),
                    (ids, "ids", (torch.int64,), 0),
                    (advanced_out, "advanced_out", (torch.uint8, torch.bool), G),
                    (wire_stats, "wire_stats", (torch.int64,), 4)))
    csr = isinstance(tracker, CsrTracker)
    if csr and ids is None:
        raise _lib.QuorumBatchError("ids (the groups' slot IDs over the tracker's off) are required")
    if not csr and rows is None and (off is None or ids is None):
        raise _lib.QuorumBatchError("rows, or off and ids, are required")
    dev = buf.device
    M = msg_group.numel()
    if reset_stats:
        tracker.stats.zero_()
    if rearm:
        tracker.stepdown_at.fill_(-1)
    lib = _lib.load()
    need = (lib.qb_wire_csr_tracker_workspace_bytes(tracker.G, tracker.max_slots, M) if csr
            else lib.qb_wire_fixed_tracker_workspace_bytes(tracker.n, tracker.G, M))
    if need == 0:
        raise _lib.QuorumBatchError(f"batch of {M} messages too large for one call")
    ws = getattr(tracker, "_wire_ws", None)
    if ws is None or ws.numel() < need:
        ws = tracker._wire_ws = torch.empty(need, dtype=torch.uint8, device=dev)
    status = torch.empty(max(M, 1), dtype=torch.uint8, device=dev)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    stream = torch.cuda.current_stream(dev).cuda_stream
    state = (p(tracker.term), p(tracker.term_start), p(tracker.match), p(tracker.next),
             p(tracker.active), p(tracker.committed), p(tracker.stepdown_at), p(advanced_out),
             status.data_ptr(), p(wire_stats), p(tracker.stats), ws.data_ptr(), ws.numel(), stream)
    if csr:
        _lib.call("qb_dev_ingest_csr_tracker_step", tracker.G, tracker.max_slots, p(tracker.off),
                  p(tracker.cfg), M, buf.data_ptr(), nbytes, msg_off.data_ptr(),
                  msg_group.data_ptr(), p(rows), p(ids), *state)
    else:
        _lib.call("qb_dev_ingest_fixed_tracker_step", tracker.n, tracker.G, M, buf.data_ptr(),
                  nbytes, msg_off.data_ptr(), msg_group.data_ptr(), p(rows), p(off), p(ids), *state)
    return status[:M]


# ------------------------------------------------------- workload synth ---

def _vfix(v: np.ndarray, n: int) -> np.ndarray:
    """Varints of exactly n bytes (v must need exactly n bytes)."""
    v = v.astype(np.uint64)
    out = np.empty((v.size, n), np.uint8)
    for k in range(n):
        b = ((v >> np.uint64(7 * k)) & np.uint64(0x7F)).astype(np.uint8)
        out[:, k] = b | (0x80 if k < n - 1 else 0)
    return out


_EMPTY_SNAPSHOT = bytes([0x12, 0x08, 0x0A, 0x02, 0x28, 0x00, 0x10, 0x00, 0x18, 0x00])
# Snapshot{Metadata{ConfState{AutoLeave:false}, Index:0, Term:0}} as gogoproto
# writes it (non-nullable fields always present).


def synth_response_stream(M: int, G: int, seed: int = 0x5EED0008, hb_frac: float = 0.1):
    """Host bytes of M gogoproto-encoded responses to G 5-voter leaders (the
    wire-ingest bench workload): MsgAppResp (10% rejected) and, with
    probability hb_frac, MsgHeartbeatResp carrying an 8-byte read context.
    Node IDs, terms and indexes are sized so every message of a kind has the
    same layout (vectorised construction).  Returns (bytes ndarray u8,
    msg_off u64 [M+1], msg_group u32 [M], off u32 [G+1], ids u64 [5G])."""
    rng = np.random.default_rng(seed)
    grp = rng.integers(0, G, M).astype(np.uint32)
    slot = rng.integers(1, 5, M).astype(np.uint64)
    g64 = grp.astype(np.uint64)
    frm = np.uint64(16384) + slot * np.uint64(200000) + (g64 % np.uint64(100000))
    to = np.uint64(16384) + (g64 % np.uint64(100000))
    term = np.full(M, 20000, np.uint64)
    index = np.uint64(1 << 35) + g64 * np.uint64(64) + rng.integers(0, 64, M).astype(np.uint64)
    reject = rng.random(M) < 0.1
    hb = rng.random(M) < hb_frac
    ctx = (np.uint64(1) << np.uint64(56)) + rng.integers(1, 1 << 40, M).astype(np.uint64)

    def col(byte):
        return np.full((M, 1), byte, np.uint8)
    app = np.concatenate([
        col(0x08), col(4), col(0x10), _vfix(to, 3), col(0x18), _vfix(frm, 3), col(0x20),
        _vfix(term, 3), col(0x28), col(0), col(0x30), _vfix(index, 6), col(0x40), col(0),
        col(0x4A), col(len(_EMPTY_SNAPSHOT)),
        np.tile(np.frombuffer(_EMPTY_SNAPSHOT, np.uint8), (M, 1)),
        col(0x50), reject.astype(np.uint8)[:, None], col(0x58), col(0)], axis=1)
    ctxb = ((ctx[:, None] >> (np.arange(7, -1, -1, dtype=np.uint64) * np.uint64(8)))
            & np.uint64(0xFF)).astype(np.uint8)
    hbm = np.concatenate([
        col(0x08), col(9), col(0x10), _vfix(to, 3), col(0x18), _vfix(frm, 3), col(0x20),
        _vfix(term, 3), col(0x28), col(0), col(0x30), col(0), col(0x40), col(0),
        col(0x4A), col(len(_EMPTY_SNAPSHOT)),
        np.tile(np.frombuffer(_EMPTY_SNAPSHOT, np.uint8), (M, 1)),
        col(0x50), col(0), col(0x58), col(0), col(0x62), col(8), ctxb], axis=1)
    la, lh = app.shape[1], hbm.shape[1]
    lens = np.where(hb, lh, la).astype(np.uint64)
    moff = np.zeros(M + 1, np.uint64)
    np.cumsum(lens, out=moff[1:])
    buf = np.empty(int(moff[-1]), np.uint8)
    for sel, t, L_ in ((~hb, app, la), (hb, hbm, lh)):
        pos = moff[:-1][sel].astype(np.int64)
        buf[(pos[:, None] + np.arange(L_)).reshape(-1)] = t[sel].reshape(-1)
    off = (np.arange(G + 1, dtype=np.uint32) * 5).astype(np.uint32)
    gg = np.repeat(np.arange(G, dtype=np.uint64), 5)
    ss = np.tile(np.arange(5, dtype=np.uint64), G)
    ids = np.uint64(16384) + ss * np.uint64(200000) + (gg % np.uint64(100000))
    return buf, moff, grp, off, ids


def _dev_varint(v: torch.Tensor, n: int) -> list:
    """Varint bytes (exactly n) of an int64 device tensor, one u8 column each."""
    cols = []
    for k in range(n):
        b = (v >> (7 * k)) & 0x7F
        if k < n - 1:
            b = b | 0x80
        cols.append(b.to(torch.uint8))
    return cols


def encode_appresp(to: torch.Tensor, frm: torch.Tensor, term: torch.Tensor,
                   index: torch.Tensor, reject: torch.Tensor):
    """Device-side gogoproto encoding of M MsgAppResp messages with one fixed
    layout (raft.pb.go Message.Marshal field order: Type, To, From, Term,
    LogTerm 0, Index, Commit 0, the empty non-nullable Snapshot, Reject,
    RejectHint 0) — the composed wire -> tracker workload's generator.  Node
    IDs and terms must need 3-byte varints ([2^14, 2^21)), indexes 6-byte
    ones ([2^35, 2^42)).  Returns (bytes u8, nbytes, msg_off int64 [M+1])."""
    lo, hi = 1 << 14, 1 << 21
    for t, what, a, b in ((to, "to", lo, hi), (frm, "frm", lo, hi), (term, "term", lo, hi),
                          (index, "index", 1 << 35, 1 << 42)):
        if t.numel() and (int(t.min()) < a or int(t.max()) >= b):
            raise ValueError(f"encode_appresp: {what} outside [{a}, {b})")
    M = to.numel()
    dev = to.device

    def col(byte):
        return torch.full((M,), byte, dtype=torch.uint8, device=dev)
    cols = [col(0x08), col(4), col(0x10), *_dev_varint(to, 3), col(0x18), *_dev_varint(frm, 3),
            col(0x20), *_dev_varint(term, 3), col(0x28), col(0), col(0x30),
            *_dev_varint(index, 6), col(0x40), col(0), col(0x4A), col(len(_EMPTY_SNAPSHOT))]
    cols += [col(b) for b in _EMPTY_SNAPSHOT]
    cols += [col(0x50), reject.to(torch.uint8), col(0x58), col(0)]
    L = len(cols)
    buf = torch.stack(cols, dim=1).reshape(-1)
    moff = torch.arange(M + 1, dtype=torch.int64, device=dev) * L
    return buf, M * L, moff
