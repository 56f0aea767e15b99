"""The leader inbox step (include/quorum_batch.h ``qb_dev_leader_step``).

Device-resident leader state of G raft groups — Progress per slot (CSR, as
``CsrGroups``), the leader's log view, the pending ReadIndex queue — and a
batch of responses applied with the reference's sequential semantics
(raft.go:847-921 Step's term filter, raft.go:1099-1342 stepLeader).  Every
computation runs in the HIP library; torch only holds device memory.

Array names and meanings (all numpy dtypes little-endian):
  off[G+1] u32, cfg[G] u32 (mask_in | mask_out << 16), meta[G] u32 (leader
  slot | transferee << 8 | runs << 16 | readq length << 20 | pending-read bit
  25), term/committed/first_index/last_index/snap_index/snap_term/max_ents[G]
  u64, run_start/run_term[8*G] u64 (run-major: run r of group g at r*G+g), match/next/pending_snapshot[S] u64,
  pstate[S] u8 (state | ProbeSent 0x4 | RecentActive 0x8), infl_pos[S] u32
  (start | count << 16), infl_buf[S*inflight_cap] u64, rq_ctx/rq_index
  [G*readq_cap] u64, rq_meta[G*readq_cap] u32 (acks | from << 16).
"""
from __future__ import annotations

import ctypes as C
import operator
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from .. import _lib
from ._checks import I32, I64, U8, check_tensors

MAX_RUNS = 8
MAX_READQ = 16

IN_APP_RESP, IN_HEARTBEAT_RESP, IN_SNAP_STATUS, IN_UNREACHABLE = 0, 1, 2, 3
PR_PROBE_SENT, PR_RECENT_ACTIVE = 0x04, 0x08
META_PENDING_READINDEX = 1 << 25
READ_ONLY_SAFE, READ_ONLY_LEASE_BASED = 0, 1
LFLAG_ADVANCED, LFLAG_RELEASE_READS, LFLAG_STEPPED_DOWN = 0x1, 0x2, 0x4
LSTAT_NAMES = ("applied", "stale_term", "higher_term", "non_member", "after_stepdown",
               "bad_group", "msgs", "msgs_dropped")

MSG_DTYPE = np.dtype([("index", "<u8"), ("log_term", "<u8"), ("commit", "<u8"), ("aux", "<u8"),
                      ("group", "<u4"), ("to", "u1"), ("type", "u1"), ("reserved", "<u2")])
assert MSG_DTYPE.itemsize == 40
# struct qb_read_state: a local read's answer (raft.go:1737-1745 ReadState)
READ_STATE_DTYPE = np.dtype([("index", "<u8"), ("ctx", "<u8")])

_P = C.c_void_p


class LeaderGroupsC(C.Structure):
    """struct qb_leader_groups (include/quorum_batch.h)."""
    _fields_ = [("G", C.c_uint64), ("inflight_cap", C.c_uint32), ("readq_cap", C.c_uint32),
                ("read_only", C.c_uint32), ("options", C.c_uint32)] + [
        (n, _P) for n in ("off", "cfg", "meta", "term", "committed", "first_index", "last_index",
                          "snap_index", "snap_term", "max_ents", "run_start", "run_term", "match",
                          "next", "pending_snapshot", "pstate", "infl_pos", "infl_buf", "rq_ctx",
                          "rq_index", "rq_meta")]


OUTBOX_SLOTS = 8    # QB_LEADER_OUTBOX_SLOTS
OUTBOX_CHUNK = 32   # QB_LEADER_OUTBOX_CHUNK


class LeaderOutboxC(C.Structure):
    """struct qb_leader_outbox (include/quorum_batch.h)."""
    _fields_ = [("slots", _P), ("count", _P), ("chunk_head", _P), ("chunk_next", _P),
                ("chunks", _P), ("nchunks", C.c_uint64), ("chunks_used", _P),
                ("read_states", _P), ("read_count", _P)]


class LeaderInboxC(C.Structure):
    """struct qb_leader_inbox."""
    _fields_ = [("M", C.c_uint64)] + [(n, _P) for n in ("group", "flags", "index", "term", "hint",
                                                         "log_term")]


GROUP_ARRAYS = {  # name -> numpy dtype (device storage uses the same bytes)
    "off": np.uint32, "cfg": np.uint32, "meta": np.uint32, "term": np.uint64,
    "committed": np.uint64, "first_index": np.uint64, "last_index": np.uint64,
    "snap_index": np.uint64, "snap_term": np.uint64, "max_ents": np.uint64,
    "run_start": np.uint64, "run_term": np.uint64, "match": np.uint64, "next": np.uint64,
    "pending_snapshot": np.uint64, "pstate": np.uint8, "infl_pos": np.uint32,
    "infl_buf": np.uint64, "rq_ctx": np.uint64, "rq_index": np.uint64, "rq_meta": np.uint32,
}
_TORCH = {np.uint8: torch.uint8, np.uint32: torch.int32, np.uint64: torch.int64,
          np.uint16: torch.int16}
_SIGNED = {np.uint8: np.uint8, np.uint32: np.int32, np.uint64: np.int64, np.uint16: np.int16}


def _to_dev(a: np.ndarray, dt, device) -> torch.Tensor:
    a = np.ascontiguousarray(np.asarray(a, dtype=dt))
    if a.size == 0:
        a = np.zeros(1, dtype=dt)  # keep a valid device pointer
    return torch.from_numpy(a.view(_SIGNED[dt]).copy()).to(device)


def _to_np(t: torch.Tensor, dt, n: Optional[int] = None) -> np.ndarray:
    a = t.detach().cpu().numpy().view(dt)
    return a if n is None else a[:n]


@dataclass
class LeaderInbox:
    """A batch of responses to leaders (SoA).  flags = slot | kind << 4 |
    0x80 if Reject; index = Message.Index (MsgHeartbeatResp: Context)."""
    group: torch.Tensor
    flags: torch.Tensor
    index: torch.Tensor
    term: torch.Tensor
    hint: torch.Tensor
    log_term: torch.Tensor

    _m: int = 0  # number of records (device arrays hold at least one element)

    @property
    def M(self) -> int:
        return self._m

    def check(self) -> None:
        """Every column a contiguous device tensor of its dtype holding M
        records (M = ``_m``, set by whoever filled the columns)."""
        try:
            M = operator.index(self._m)
        except TypeError:
            M = -1
        if M < 0:
            raise _lib.QuorumBatchError(f"inbox record count must be a non-negative int, "
                                        f"got {self._m!r}")
        check_tensors(((self.group, "inbox.group", I32, M), (self.flags, "inbox.flags", U8, M),
                       (self.index, "inbox.index", I64, M), (self.term, "inbox.term", I64, M),
                       (self.hint, "inbox.hint", I64, M),
                       (self.log_term, "inbox.log_term", I64, M)))

    @classmethod
    def from_numpy(cls, group, slot, kind, index, term, reject=None, hint=None, log_term=None,
                   device="cuda"):
        dev = torch.device(device)
        M = len(group)
        flags = (np.asarray(slot, np.uint8) & 0x0F) | ((np.asarray(kind, np.uint8) & 3) << 4)
        if reject is not None:
            flags = flags | (np.asarray(reject, bool).astype(np.uint8) << 7)
        z = np.zeros(M, np.uint64)
        ib = cls(_to_dev(np.asarray(group, np.uint32), np.uint32, dev),
                 _to_dev(flags.astype(np.uint8), np.uint8, dev),
                 _to_dev(index, np.uint64, dev), _to_dev(term, np.uint64, dev),
                 _to_dev(z if hint is None else hint, np.uint64, dev),
                 _to_dev(z if log_term is None else log_term, np.uint64, dev))
        ib._m = M
        return ib


@dataclass
class LeaderStepResult:
    msgs: np.ndarray        # MSG_DTYPE, group order
    msg_total: int
    msg_off: np.ndarray     # [G+1] u32
    stepdown_at: np.ndarray  # [G] u32 (0xFFFFFFFF = none)
    gflags: np.ndarray      # [G] u8
    stats: Dict[str, int]
    # step_outbox(read_states=True): the local reads' answers, group order
    # (Ready.ReadStates), and each group's first; else None
    read_states: Optional[np.ndarray] = None  # READ_STATE_DTYPE
    read_off: Optional[np.ndarray] = None     # [G+1]


class LeaderGroups:
    """Leader state of G groups resident on one device."""

    options = 0  # QB_LEADER_OPT_* (diagnostic switches)

    def __init__(self, arrays: Dict[str, np.ndarray], inflight_cap: int, readq_cap: int = 0,
                 read_only: int = READ_ONLY_SAFE, device="cuda"):
        self.device = torch.device(device)
        self.G = len(arrays["cfg"])
        self.S = int(arrays["off"][-1]) if len(arrays["off"]) else 0
        self.inflight_cap, self.readq_cap, self.read_only = inflight_cap, readq_cap, read_only
        need = self._lengths()
        for k in GROUP_ARRAYS:
            if k not in arrays:
                raise _lib.QuorumBatchError(f"leader state array {k!r} missing")
            if np.asarray(arrays[k]).size < need[k]:
                raise _lib.QuorumBatchError(f"leader state array {k!r} holds "
                                            f"{np.asarray(arrays[k]).size} entries, < {need[k]}")
        if not 1 <= inflight_cap <= 4096:
            raise _lib.QuorumBatchError(f"inflight_cap must be 1..4096, got {inflight_cap}")
        # the rings' invariant (start < cap, count <= cap): the step indexes a
        # slot's ring by it without a check (include/quorum_batch.h)
        ip = np.asarray(arrays["infl_pos"]).astype(np.uint32)[: self.S]
        bad = ((ip & 0xFFFF) >= inflight_cap) | ((ip >> 16) > inflight_cap)
        if bad.any():
            j = int(np.argmax(bad))
            raise _lib.QuorumBatchError(f"infl_pos[{j}] = {int(ip[j]):#x} breaks the ring invariant "
                                        f"(start < {inflight_cap}, count <= {inflight_cap})")
        if not self.device.type == "cuda":
            raise _lib.QuorumBatchError("LeaderGroups needs a HIP device; there is no CPU path")
        self.t = {k: _to_dev(arrays[k], dt, self.device) for k, dt in GROUP_ARRAYS.items()}
        self._ws = None

    def _lengths(self) -> Dict[str, int]:
        """Entries per state array (include/quorum_batch.h qb_leader_groups)."""
        return {"off": self.G + 1, "cfg": self.G, "meta": self.G, "term": self.G,
             "committed": self.G, "first_index": self.G, "last_index": self.G,
             "snap_index": self.G, "snap_term": self.G, "max_ents": self.G,
             "run_start": self.G * MAX_RUNS, "run_term": self.G * MAX_RUNS,
             "match": self.S, "next": self.S, "pending_snapshot": self.S, "pstate": self.S,
             "infl_pos": self.S, "infl_buf": self.S * self.inflight_cap,
             "rq_ctx": self.G * self.readq_cap, "rq_index": self.G * self.readq_cap,
             "rq_meta": self.G * self.readq_cap}

    def numpy(self) -> Dict[str, np.ndarray]:
        n = self._lengths()
        return {k: _to_np(self.t[k], dt, n[k]) for k, dt in GROUP_ARRAYS.items()}

    def _struct(self) -> LeaderGroupsC:
        s = LeaderGroupsC(G=self.G, inflight_cap=self.inflight_cap, readq_cap=self.readq_cap,
                          read_only=self.read_only, options=self.options)
        for k in GROUP_ARRAYS:
            setattr(s, k, self.t[k].data_ptr())
        return s

    def step(self, inbox: LeaderInbox, msg_cap: Optional[int] = None,
             stats: Optional[torch.Tensor] = None, fetch: bool = True):
        """One batch through qb_dev_leader_step.  Returns a LeaderStepResult
        (host copies) when fetch, else the device outputs."""
        inbox.check()
        check_tensors(((stats, "stats", I64, len(LSTAT_NAMES)),))
        lib = _lib.load()
        M = inbox.M
        dev = self.device
        need = lib.qb_leader_workspace_bytes(self.G, M)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=dev)
        if msg_cap is None:
            msg_cap = max(16, 8 * M + 4 * self.G)
        out = self._outputs(msg_cap)
        if stats is None:
            stats = torch.zeros(8, dtype=torch.int64, device=dev)
        ls = self._struct()
        ib = LeaderInboxC(M=M, group=inbox.group.data_ptr(), flags=inbox.flags.data_ptr(),
                          index=inbox.index.data_ptr(), term=inbox.term.data_ptr(),
                          hint=inbox.hint.data_ptr(), log_term=inbox.log_term.data_ptr())
        _lib.call("qb_dev_leader_step", C.byref(ls), C.byref(ib), out["msgs"].data_ptr(), msg_cap,
                  out["total"].data_ptr(), out["off"].data_ptr(), out["stepdown"].data_ptr(),
                  out["gflags"].data_ptr(), stats.data_ptr(), self._ws.data_ptr(),
                  self._ws.numel(), torch.cuda.current_stream(dev).cuda_stream)
        if not fetch:
            return out, stats
        total = int(out["total"].cpu().item())
        raw = out["msgs"].cpu().numpy().view(np.uint8)[: min(total, msg_cap) * 40]
        st = stats.cpu().tolist()
        return LeaderStepResult(
            msgs=raw.view(MSG_DTYPE).copy(), msg_total=total,
            msg_off=_to_np(out["off"], np.uint32, self.G + 1),
            stepdown_at=_to_np(out["stepdown"], np.uint32, self.G),
            gflags=_to_np(out["gflags"], np.uint8, self.G),
            stats={k: st[i] for i, k in enumerate(LSTAT_NAMES)})

    def step_outbox(self, inbox: LeaderInbox, nchunks: Optional[int] = None,
                    stats: Optional[torch.Tensor] = None, fetch: bool = True,
                    read_states: bool = False):
        """One batch through qb_dev_leader_step_outbox: the messages stay in
        the per-group outbox (8 k-major slots per group + 32-message overflow
        chunks) the step writes them to.  read_states: the local reads'
        answers go to the outbox's ReadState area (readq_cap k-major rows)
        instead of the messages, as the reference's r.readStates.  fetch: a
        LeaderStepResult with the outbox read back into group order on the
        host (msg_total = messages stored); else the device outbox dict and
        stats."""
        inbox.check()
        check_tensors(((stats, "stats", I64, len(LSTAT_NAMES)),))
        lib = _lib.load()
        M, G, dev = inbox.M, self.G, self.device
        need = lib.qb_leader_outbox_workspace_bytes(G, M)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=dev)
        if nchunks is None:
            nchunks = M // 8 + 1024
        ob = self._outbox(nchunks, read_states)
        if stats is None:
            stats = torch.zeros(8, dtype=torch.int64, device=dev)
        ls = self._struct()
        ib = LeaderInboxC(M=M, group=inbox.group.data_ptr(), flags=inbox.flags.data_ptr(),
                          index=inbox.index.data_ptr(), term=inbox.term.data_ptr(),
                          hint=inbox.hint.data_ptr(), log_term=inbox.log_term.data_ptr())
        oc = LeaderOutboxC(slots=ob["slots"].data_ptr(), count=ob["count"].data_ptr(),
                           chunk_head=ob["chunk_head"].data_ptr(),
                           chunk_next=ob["chunk_next"].data_ptr() if nchunks else None,
                           chunks=ob["chunks"].data_ptr() if nchunks else None, nchunks=nchunks,
                           chunks_used=ob["chunks_used"].data_ptr(),
                           read_states=ob["read_states"].data_ptr() if read_states else None,
                           read_count=ob["read_count"].data_ptr() if read_states else None)
        _lib.call("qb_dev_leader_step_outbox", C.byref(ls), C.byref(ib), C.byref(oc),
                  ob["stepdown"].data_ptr(), ob["gflags"].data_ptr(), stats.data_ptr(),
                  self._ws.data_ptr(), self._ws.numel(), torch.cuda.current_stream(dev).cuda_stream)
        if not fetch:
            return ob, stats
        return self.fetch_outbox(ob, stats, nchunks)

    def fetch_outbox(self, ob, stats, nchunks: int) -> "LeaderStepResult":
        """The device outbox of a step_outbox(..., fetch=False) call read back
        into group order on the host (a LeaderStepResult)."""
        G = self.G
        cnt = _to_np(ob["count"], np.uint32, G).astype(np.int64)
        slots = ob["slots"].cpu().numpy().view(MSG_DTYPE).reshape(OUTBOX_SLOTS, G)
        chunks = ob["chunks"].cpu().numpy().view(MSG_DTYPE) if nchunks else None
        head = _to_np(ob["chunk_head"], np.uint32, G)
        nxt = _to_np(ob["chunk_next"], np.uint32, nchunks) if nchunks else None
        off = np.zeros(G + 1, np.int64)
        off[1:] = np.cumsum(cnt)
        msgs = np.empty(int(off[-1]), MSG_DTYPE)
        for k in range(OUTBOX_SLOTS):        # row k of every group with > k messages
            sel = np.nonzero(cnt > k)[0]
            msgs[off[sel] + k] = slots[k, sel]
        # the overflow chains, one chunk level at a time over every group
        # whose chain reaches it (vectorised: a hot batch gives many groups
        # hundreds of messages each)
        sel = np.nonzero(cnt > OUTBOX_SLOTS)[0]
        c = head[sel].astype(np.int64)
        j0 = 0
        while sel.size:
            n_here = np.minimum(cnt[sel] - OUTBOX_SLOTS - j0, OUTBOX_CHUNK)
            for k in range(OUTBOX_CHUNK):
                m = n_here > k
                if not m.any():
                    break
                msgs[off[sel[m]] + OUTBOX_SLOTS + j0 + k] = chunks[c[m] * OUTBOX_CHUNK + k]
            j0 += OUTBOX_CHUNK
            more = cnt[sel] > OUTBOX_SLOTS + j0
            sel = sel[more]
            if sel.size:
                c = nxt[c[more]].astype(np.int64)
        st = stats.cpu().tolist()
        rs = roff = None
        if "read_states" in ob:
            rcnt = _to_np(ob["read_count"], np.uint32, G).astype(np.int64)
            rows = ob["read_states"].cpu().numpy().view(READ_STATE_DTYPE).reshape(-1, G)
            roff = np.zeros(G + 1, np.int64)
            roff[1:] = np.cumsum(rcnt)
            rs = np.empty(int(roff[-1]), READ_STATE_DTYPE)
            for k in range(rows.shape[0]):
                sel = np.nonzero(rcnt > k)[0]
                rs[roff[sel] + k] = rows[k, sel]
        return LeaderStepResult(
            msgs=msgs, msg_total=int(off[-1]), msg_off=off.astype(np.uint32),
            stepdown_at=_to_np(ob["stepdown"], np.uint32, G),
            gflags=_to_np(ob["gflags"], np.uint8, G),
            stats={k: st[i] for i, k in enumerate(LSTAT_NAMES)},
            read_states=rs, read_off=roff)

    def _outbox(self, nchunks: int, read_states: bool = False):
        dev, G = self.device, self.G
        key = ("outbox", nchunks, read_states)
        if getattr(self, "_ob_key", None) != key:
            self._ob = {"slots": torch.empty(OUTBOX_SLOTS * G * 40, dtype=torch.uint8, device=dev),
                        "count": torch.zeros(G, dtype=torch.int32, device=dev),
                        "chunk_head": torch.zeros(G, dtype=torch.int32, device=dev),
                        "chunk_next": torch.zeros(max(nchunks, 1), dtype=torch.int32, device=dev),
                        "chunks": torch.empty(max(nchunks, 1) * OUTBOX_CHUNK * 40, dtype=torch.uint8,
                                              device=dev),
                        "chunks_used": torch.zeros(1, dtype=torch.int32, device=dev),
                        "stepdown": torch.zeros(G, dtype=torch.int32, device=dev),
                        "gflags": torch.zeros(G, dtype=torch.uint8, device=dev)}
            if read_states:
                self._ob["read_states"] = torch.empty(max(self.readq_cap, 1) * G * 16,
                                                      dtype=torch.uint8, device=dev)
                self._ob["read_count"] = torch.zeros(G, dtype=torch.int32, device=dev)
            self._ob_key = key
        return self._ob

    def _outputs(self, msg_cap: int):
        dev = self.device
        key = (msg_cap,)
        if getattr(self, "_out_key", None) != key:
            self._out = {"msgs": torch.empty(msg_cap * 40, dtype=torch.uint8, device=dev),
                         "total": torch.zeros(1, dtype=torch.int64, device=dev),
                         "off": torch.zeros(self.G + 1, dtype=torch.int32, device=dev),
                         "stepdown": torch.zeros(self.G, dtype=torch.int32, device=dev),
                         "gflags": torch.zeros(self.G, dtype=torch.uint8, device=dev)}
            self._out_key = key
        return self._out


# ------------------------------------------------------- workload synth ---

def synth_streaming(G: int, W: int = 32, D: int = 4, n: int = 5, device="cuda"):
    """Steady-state leaders (bench/test workload of the leader step: 5 voters, leader slot
    0, every follower Replicate with a full window of W in-flight MsgApps of D
    entries each (MaxInflightMsgs = W), commit at the window base."""
    dev = torch.device(device)
    g = torch.arange(G, dtype=torch.int64, device=dev)
    base = 1000 + (g * 37) % 1000
    last = base + W * D
    S = n * G
    lg = LeaderGroups.__new__(LeaderGroups)
    lg.device, lg.G, lg.S = dev, G, S
    lg.inflight_cap, lg.readq_cap, lg.read_only, lg._ws = W, 0, 0, None
    i32 = lambda x: x.to(torch.int32)
    runs = torch.zeros(G * MAX_RUNS, dtype=torch.int64, device=dev)
    runs_t = torch.zeros_like(runs)
    runs[:G] = base - 51  # run 0 of every group (run-major)
    runs_t[:G] = 7
    slot = torch.arange(S, dtype=torch.int64, device=dev) % n
    gs = torch.arange(S, dtype=torch.int64, device=dev) // n
    bs, ls = base[gs], last[gs]
    lead = slot == 0
    j = torch.arange(W, dtype=torch.int64, device=dev)
    infl = (bs[:, None] + (j[None, :] + 1) * D).reshape(-1)
    lg.t = {
        "off": i32(torch.arange(0, S + 1, n, device=dev)),
        "cfg": torch.full((G,), (1 << n) - 1, dtype=torch.int32, device=dev),
        "meta": torch.full((G,), 0xFF00 | (1 << 16), dtype=torch.int32, device=dev),
        "term": torch.full((G,), 7, dtype=torch.int64, device=dev),
        "committed": base.clone(), "first_index": base - 50, "last_index": last,
        "snap_index": base - 51, "snap_term": torch.full((G,), 7, dtype=torch.int64, device=dev),
        "max_ents": torch.full((G,), D, dtype=torch.int64, device=dev),
        "run_start": runs, "run_term": runs_t,
        "match": torch.where(lead, ls, bs), "next": ls + 1,
        "pending_snapshot": torch.zeros(S, dtype=torch.int64, device=dev),
        "pstate": torch.full((S,), 1 | 8, dtype=torch.uint8, device=dev),
        "infl_pos": i32(torch.where(lead, torch.zeros_like(slot), torch.full_like(slot, W << 16))),
        "infl_buf": infl,
        "rq_ctx": torch.zeros(1, dtype=torch.int64, device=dev),
        "rq_index": torch.zeros(1, dtype=torch.int64, device=dev),
        "rq_meta": torch.zeros(1, dtype=torch.int32, device=dev),
    }
    return lg, base


def streaming_inbox(G: int, base: torch.Tensor, k: int, D: int = 4, n: int = 5, device="cuda",
                    shuffle: bool = True):
    """Step k: one MsgAppResp per group, from follower 1 + (g + k) % 4, acking
    the next window boundary; records shuffled (arrival order) unless
    ``shuffle`` is False (records already in group order)."""
    dev = torch.device(device)
    g = torch.randperm(G, device=dev) if shuffle else torch.arange(G, device=dev)
    f = 1 + (g + k) % (n - 1)
    idx = base[g] + (k // (n - 1) + 1) * D
    z = torch.zeros(G, dtype=torch.int64, device=dev)
    ib = LeaderInbox(g.to(torch.int32), f.to(torch.uint8), idx, torch.full_like(idx, 7), z, z)
    ib._m = G
    return ib


def synth_readindex(G: int, Q: int = 4, n: int = 5, device="cuda"):
    """Caught-up leaders (5 voters, every follower Replicate at the last
    index) each holding Q pending ReadIndex requests (read_only.go:30-40: the
    leader's own ack recorded, request contexts ctx0 + g*Q + k, half of them
    from a follower, half local) — the ReadIndex / CheckQuorum bench workload
    of SURVEY.md §8f row 2.  Returns (LeaderGroups, pristine read-queue
    tensors to restore before each step)."""
    lg, base = synth_streaming(G, W=4, D=1, n=n, device=device)
    dev = torch.device(device)
    S = n * G
    last = lg.t["last_index"]
    slot = torch.arange(S, dtype=torch.int64, device=dev) % n
    gs = torch.arange(S, dtype=torch.int64, device=dev) // n
    lg.t["match"] = last[gs].clone()
    lg.t["next"] = last[gs] + 1
    lg.t["committed"] = last.clone()
    lg.t["infl_pos"] = torch.zeros(S, dtype=torch.int32, device=dev)
    lg.readq_cap = Q
    g = torch.arange(G, dtype=torch.int64, device=dev)
    k = torch.arange(Q, dtype=torch.int64, device=dev)
    ctx = ((1 << 40) + g[:, None] * Q + k[None, :]).reshape(-1)
    idx = last[:, None].expand(G, Q).reshape(-1).clone()
    frm = torch.where(k % 2 == 0, torch.full_like(k, 0xFF), 1 + (k % (n - 1)))
    meta = (1 | (frm[None, :].expand(G, Q) << 16)).reshape(-1).to(torch.int32)  # leader acked
    lg.t["rq_ctx"], lg.t["rq_index"], lg.t["rq_meta"] = ctx, idx, meta
    lg.t["meta"] = torch.full((G,), 0xFF00 | (1 << 16) | (Q << 20), dtype=torch.int32, device=dev)
    pristine = {k_: lg.t[k_].clone() for k_ in ("rq_ctx", "rq_index", "rq_meta", "meta")}
    return lg, ctx.view(G, Q)[:, Q - 1].clone(), pristine


def readindex_inbox(G: int, last_ctx: torch.Tensor, n: int = 5, device="cuda"):
    """Two heartbeat responses per group (followers 1 and 2, shuffled arrival)
    carrying the latest request context: the second one completes the quorum
    and releases all Q requests (read_only.go:84-121)."""
    dev = torch.device(device)
    g = torch.randperm(2 * G, device=dev) % G
    # follower 1 for a group's first record, follower 2 for its second
    order = torch.argsort(g, stable=True)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(2 * G, device=dev) % 2
    f = (1 + rank).to(torch.uint8) | (1 << 4)  # kind MsgHeartbeatResp
    z = torch.zeros(2 * G, dtype=torch.int64, device=dev)
    ib = LeaderInbox(g.to(torch.int32), f.to(torch.uint8), last_ctx[g],
                     torch.full((2 * G,), 7, dtype=torch.int64, device=dev), z, z)
    ib._m = 2 * G
    return ib
