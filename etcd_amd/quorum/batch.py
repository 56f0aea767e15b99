"""raft/quorum/batch — the batch engine's Python face.

Mirror of the Go ``raft/quorum/batch`` package that INTEGRATION.md describes:
G independent raft groups evaluated per call, state resident in HBM as
structure-of-arrays, every computation a HIP kernel behind the C ABI
(include/quorum_batch.h).  torch is used only for device memory, streams and
host<->device copies.

Device tensors hold uint64 values in int64 storage (bit-identical); use
``as_u64`` to view them as numpy uint64 after ``.cpu()``.

Reference semantics (paths relative to the reference's raft/):
  MajorityConfig.CommittedIndex / VoteResult   quorum/majority.go:126-210
  JointConfig.CommittedIndex / VoteResult      quorum/joint.go:49-75
  ProgressTracker.QuorumActive                 tracker/tracker.go:215-225
  Progress.MaybeUpdate                         tracker/progress.go:144-153
  raft.maybeCommit -> raftLog.maybeCommit      raft.go:585-588, log.go:328-334
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from .. import _lib
from ._checks import FLAG, I16, I32, I64, U8, check_tensors

INDEX_INF = (1 << 64) - 1


def as_u64(t: torch.Tensor) -> np.ndarray:
    """View an int64 tensor (device or host) as numpy uint64."""
    return t.detach().cpu().numpy().view(np.uint64)


def from_u64(a, device) -> torch.Tensor:
    """numpy uint64 (or anything np.asarray accepts) -> int64 tensor on device."""
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.uint64)).view(np.int64)
    return torch.from_numpy(arr.copy()).to(device)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check_outs(G: int, commit_out, vote_out) -> None:
    check_tensors(((commit_out, "commit_out", I64, G), (vote_out, "vote_out", U8, G)))


def mask_dtype(n: int):
    return torch.uint8 if n <= 8 else torch.int16


# ---------------------------------------------------------------- FIXED ---

class FixedGroups:
    """G groups sharing one n-voter MajorityConfig shape (FIXED layout).

    ``match`` is [n, G] (slot-major), ``voted``/``granted`` are per-group slot
    bitmasks (uint8 for n <= 8, int16 bits for n <= 16).
    """

    def __init__(self, n: int, G: int, device="cuda", match=None, voted=None, granted=None):
        if not 0 <= n <= _lib.QB_MAX_SLOTS:
            raise ValueError(f"n must be 0..{_lib.QB_MAX_SLOTS}")
        self.n, self.G, self.device = n, G, torch.device(device)
        mt = mask_dtype(n)
        self.match = match if match is not None else torch.zeros((n, G), dtype=torch.int64,
                                                                  device=self.device)
        self.voted = voted if voted is not None else torch.zeros(G, dtype=mt, device=self.device)
        self.granted = granted if granted is not None else torch.zeros(G, dtype=mt,
                                                                       device=self.device)
        check_tensors(((self.match, "match", I64, n * G), (self.voted, "voted", (mt,), G),
                       (self.granted, "granted", (mt,), G)))

    @classmethod
    def synth(cls, seed: int, n: int, G: int, g_begin: int = 0, device="cuda",
              with_term_start: bool = False):
        """Counter-based synthetic groups (qb_dev_synth_fixed)."""
        fg = cls(n, G, device, match=torch.empty((n, G), dtype=torch.int64, device=device),
                 voted=torch.empty(G, dtype=mask_dtype(n), device=device),
                 granted=torch.empty(G, dtype=mask_dtype(n), device=device))
        ts = torch.empty(G, dtype=torch.int64, device=device) if with_term_start else None
        _lib.call("qb_dev_synth_fixed", seed, n, G, g_begin, _ptr(fg.match), _ptr(fg.voted),
                  _ptr(fg.granted), _ptr(ts), _stream(fg.device))
        fg.term_start = ts
        return fg

    def committed_vote(self, commit_out: Optional[torch.Tensor] = None,
                       vote_out: Optional[torch.Tensor] = None, want_commit=True, want_vote=True):
        """Enqueue CommittedIndex and/or VoteResult for all G groups."""
        if want_commit and commit_out is None:
            commit_out = torch.empty(self.G, dtype=torch.int64, device=self.device)
        if want_vote and vote_out is None:
            vote_out = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        _check_outs(self.G, commit_out if want_commit else None, vote_out if want_vote else None)
        _lib.call("qb_dev_fixed_committed_vote", self.n, self.G, _ptr(self.match),
                  _ptr(self.voted), _ptr(self.granted), _ptr(commit_out if want_commit else None),
                  _ptr(vote_out if want_vote else None), _stream(self.device))
        return (commit_out if want_commit else None), (vote_out if want_vote else None)

    def committed_index(self) -> torch.Tensor:
        return self.committed_vote(want_vote=False)[0]

    def vote_result(self) -> torch.Tensor:
        return self.committed_vote(want_commit=False)[1]


# ------------------------------------------------------------------ CSR ---

@dataclass
class CompiledConfigs:
    """Host-side result of compiling per-group configs to the CSR layout.

    slot ids per group are the sorted union of Voters[0], Voters[1] and the
    learners (MajorityConfig.Slice order, majority.go:106-113)."""
    off: np.ndarray       # uint32 [G+1]
    cfg: np.ndarray       # uint32 [G]  mask_in | mask_out << 16
    slot_ids: np.ndarray  # uint64 [off[G]]

    @property
    def G(self) -> int:
        return len(self.cfg)

    def slots(self, g: int) -> np.ndarray:
        return self.slot_ids[self.off[g]:self.off[g + 1]]


def _id_csr(lists, G):
    """Per-group ID iterables -> (off uint32 [G+1], ids uint64)."""
    off = np.zeros(G + 1, dtype=np.uint32)
    flat = []
    for g, ids in enumerate(lists):
        ids = list(ids)
        off[g + 1] = off[g] + len(ids)
        flat.extend(ids)
    return off, np.asarray(flat if flat else [0], dtype=np.uint64)


def compile_configs(voters_in: Sequence[Iterable[int]], voters_out: Sequence[Iterable[int]] = None,
                    learners: Sequence[Iterable[int]] = None) -> CompiledConfigs:
    """tracker.Config (tracker.go:27-78) per group -> CSR slots and masks, by
    the C ABI's qb_host_compile_configs (the call a cgo embedder makes).

    Learners must not intersect the voters (confchange.go:307-318) and a group
    holds at most QB_MAX_SLOTS members — a violation raises ValueError with
    the reference's message."""
    G = len(voters_in)
    voters_out = voters_out if voters_out is not None else [()] * G
    learners = learners if learners is not None else [()] * G
    if len(voters_out) != G or len(learners) != G:
        raise ValueError("voters_in, voters_out and learners must have one entry per group")
    return compile_configs_csr(*_id_csr(voters_in, G), *_id_csr(voters_out, G),
                               *_id_csr(learners, G))


def compile_configs_csr(in_off, in_ids, out_off=None, out_ids=None, lrn_off=None,
                        lrn_ids=None) -> CompiledConfigs:
    """qb_host_compile_configs over ID lists already in CSR form (numpy:
    uint32 offsets [G+1], uint64 IDs)."""
    in_off = np.ascontiguousarray(in_off, np.uint32)
    G = len(in_off) - 1
    arrs = [in_off, np.ascontiguousarray(in_ids, np.uint64)]
    for o, i in ((out_off, out_ids), (lrn_off, lrn_ids)):
        arrs += [None, None] if o is None else [np.ascontiguousarray(o, np.uint32),
                                                np.ascontiguousarray(i, np.uint64)]
    ptrs = [None if a is None else a.ctypes.data for a in arrs]
    off = np.zeros(G + 1, dtype=np.uint32)
    cfg = np.zeros(max(G, 1), dtype=np.uint32)
    bad = np.zeros(1, dtype=np.uint64)
    lib = _lib.load()
    rc = lib.qb_host_compile_configs(G, *ptrs, off.ctypes.data, cfg.ctypes.data, None, 0,
                                     bad.ctypes.data)
    if rc == _lib.QB_EINVAL:
        raise ValueError(lib.qb_last_error().decode(errors="replace"))
    _lib.check(rc, "qb_host_compile_configs")
    ids = np.zeros(max(int(off[G]), 1), dtype=np.uint64)
    _lib.call("qb_host_compile_configs", G, *ptrs, off.ctypes.data, cfg.ctypes.data,
              ids.ctypes.data, ids.size, None)
    return CompiledConfigs(off, cfg[:G], ids[: int(off[G])])


@dataclass
class CompiledWide:
    """Per-slot flags layout for configs wider than 16 slots (WIDE)."""
    off: np.ndarray       # uint32 [G+1]
    flags: np.ndarray     # uint8 [off[G]]: 1 incoming, 2 outgoing (+4 voted, 8 granted)
    slot_ids: np.ndarray  # uint64 [off[G]]

    @property
    def G(self) -> int:
        return len(self.off) - 1

    def slots(self, g: int) -> np.ndarray:
        return self.slot_ids[self.off[g]:self.off[g + 1]]


def compile_configs_wide(voters_in, voters_out=None, learners=None) -> CompiledWide:
    """tracker.Config per group -> WIDE layout (any number of slots up to
    QB_WIDE_MAX_SLOTS); same slot order and learner rule as compile_configs."""
    G = len(voters_in)
    voters_out = voters_out if voters_out is not None else [()] * G
    learners = learners if learners is not None else [()] * G
    off = np.zeros(G + 1, dtype=np.uint32)
    flags, ids = [], []
    for g in range(G):
        vi, vo, lr = set(voters_in[g]), set(voters_out[g]), set(learners[g])
        if lr & (vi | vo):
            raise ValueError(f"group {g}: learners {sorted(lr & (vi | vo))} are also voters")
        slot = sorted(vi | vo | lr)
        if len(slot) > _lib.QB_WIDE_MAX_SLOTS:
            raise ValueError(f"group {g}: {len(slot)} slots > {_lib.QB_WIDE_MAX_SLOTS}")
        flags += [(1 if i in vi else 0) | (2 if i in vo else 0) for i in slot]
        ids += slot
        off[g + 1] = off[g] + len(slot)
    return CompiledWide(off, np.asarray(flags, np.uint8), np.asarray(ids, np.uint64))


class WideGroups:
    """G groups of the WIDE layout resident on one device."""

    def __init__(self, off: torch.Tensor, match: torch.Tensor, flags: torch.Tensor,
                 max_slots: Optional[int] = None):
        check_tensors(((off, "off", I32, 1), (match, "match", I64, 1), (flags, "flags", U8, 1)))
        self.off, self.match, self.flags = off, match, flags
        self.G = off.numel() - 1
        self.device = off.device
        if max_slots is None:
            max_slots = int((off[1:].long() - off[:-1].long()).max().item()) if self.G else 0
        self.max_slots = max(1, min(int(max_slots), _lib.QB_WIDE_MAX_SLOTS))

    @classmethod
    def from_compiled(cls, cw: CompiledWide, match_u64, voted=None, granted=None,
                      device="cuda"):
        """voted / granted: optional bool arrays per slot (the votes map)."""
        dev = torch.device(device)
        fl = cw.flags.copy()
        if voted is not None:
            fl |= (np.asarray(voted, bool).astype(np.uint8) << 2)
        if granted is not None:
            fl |= ((np.asarray(granted, bool) & np.asarray(voted, bool)).astype(np.uint8) << 3)
        m = np.asarray(match_u64, np.uint64)
        return cls(torch.from_numpy(cw.off.view(np.int32).copy()).to(dev),
                   from_u64(m if m.size else np.zeros(2, np.uint64), dev),
                   torch.from_numpy(fl if fl.size else np.zeros(1, np.uint8)).to(dev))

    def committed_vote(self, commit_out=None, vote_out=None, want_commit=True, want_vote=True):
        if want_commit and commit_out is None:
            commit_out = torch.empty(self.G, dtype=torch.int64, device=self.device)
        if want_vote and vote_out is None:
            vote_out = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        _check_outs(self.G, commit_out if want_commit else None, vote_out if want_vote else None)
        _lib.call("qb_dev_wide_committed_vote", self.G, self.max_slots, _ptr(self.off),
                  _ptr(self.match), _ptr(self.flags), _ptr(commit_out if want_commit else None),
                  _ptr(vote_out if want_vote else None), _stream(self.device))
        return (commit_out if want_commit else None), (vote_out if want_vote else None)


class CsrGroups:
    """G ragged / joint groups (CSR layout) resident on one device."""

    def __init__(self, off: torch.Tensor, cfg: torch.Tensor, match: torch.Tensor,
                 votes: Optional[torch.Tensor] = None, active: Optional[torch.Tensor] = None,
                 max_slots: Optional[int] = None):
        self.off, self.cfg, self.match = off, cfg, match
        self.G = cfg.numel()
        self.device = cfg.device
        if max_slots is None:  # the table's bound on s_g sizes the kernel
            max_slots = int((off[1:].long() - off[:-1].long()).max().item()) if self.G else 0
        self.max_slots = max(1, min(int(max_slots), _lib.QB_MAX_SLOTS))
        self.votes = votes if votes is not None else torch.zeros(self.G, dtype=torch.int32,
                                                                 device=self.device)
        self.active = active
        check_tensors(((off, "off", I32, self.G + 1), (cfg, "cfg", I32, self.G),
                       (match, "match", I64, 1), (self.votes, "votes", I32, self.G),
                       (active, "active", I16, self.G)))

    @classmethod
    def from_compiled(cls, cc: CompiledConfigs, match_u64: np.ndarray, votes_u32=None,
                      active_u16=None, device="cuda"):
        dev = torch.device(device)
        off = torch.from_numpy(cc.off.view(np.int32).copy()).to(dev)
        cfg = torch.from_numpy(cc.cfg.view(np.int32).copy()).to(dev)
        # keep at least one element so the pointer is valid for an all-empty batch
        m = np.asarray(match_u64, dtype=np.uint64)
        match = from_u64(m if m.size else np.zeros(2, np.uint64), dev)
        votes = None
        if votes_u32 is not None:
            votes = torch.from_numpy(np.asarray(votes_u32, np.uint32).view(np.int32).copy()).to(dev)
        active = None
        if active_u16 is not None:
            active = torch.from_numpy(np.asarray(active_u16, np.uint16).view(np.int16).copy()).to(dev)
        return cls(off, cfg, match, votes, active)

    @classmethod
    def synth(cls, seed: int, kind: str, G: int, g_begin: int = 0, device="cuda"):
        """Synthetic ragged ('ragged': 3-9 voters + 0-2 learners) or joint
        ('joint': 5+5 with overlap 0-5) groups."""
        k = {"ragged": 0, "joint": 1}[kind]
        off_h = np.empty(G + 1, dtype=np.uint32)
        fn = "qb_host_synth_csr_offsets" if k == 0 else "qb_host_synth_joint_offsets"
        _lib.call(fn, seed, G, g_begin, off_h.ctypes.data)
        dev = torch.device(device)
        off = torch.from_numpy(off_h.view(np.int32)).to(dev)
        total = int(off_h[-1])
        match = torch.empty(max(total, 2), dtype=torch.int64, device=dev)
        cfg = torch.empty(G, dtype=torch.int32, device=dev)
        votes = torch.empty(G, dtype=torch.int32, device=dev)
        _lib.call("qb_dev_synth_csr", seed, k, G, g_begin, _ptr(off), _ptr(match), _ptr(cfg),
                  _ptr(votes), _stream(dev))
        smax = int(np.diff(off_h.astype(np.int64)).max()) if G else 0
        return cls(off, cfg, match, votes, max_slots=smax)

    def committed_vote(self, commit_out=None, vote_out=None, want_commit=True, want_vote=True,
                       validate: bool = False):
        """JointConfig.CommittedIndex / VoteResult for every group.  validate:
        check the table first (qb_dev_csr_committed_vote_checked; synchronises)
        and raise QuorumBatchError on a table breaking its max_slots bound."""
        if want_commit and commit_out is None:
            commit_out = torch.empty(self.G, dtype=torch.int64, device=self.device)
        if want_vote and vote_out is None:
            vote_out = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        _check_outs(self.G, commit_out if want_commit else None, vote_out if want_vote else None)
        args = (self.G, self.max_slots, _ptr(self.off), _ptr(self.match), _ptr(self.cfg),
                _ptr(self.votes), _ptr(commit_out if want_commit else None),
                _ptr(vote_out if want_vote else None))
        if validate:
            bad = torch.empty(1, dtype=torch.int64, device=self.device)
            _lib.call("qb_dev_csr_committed_vote_checked", *args, _ptr(bad), _stream(self.device))
        else:
            _lib.call("qb_dev_csr_committed_vote", *args, _stream(self.device))
        return (commit_out if want_commit else None), (vote_out if want_vote else None)

    def committed_index(self) -> torch.Tensor:
        return self.committed_vote(want_vote=False)[0]

    def vote_result(self) -> torch.Tensor:
        return self.committed_vote(want_commit=False)[1]

    def quorum_active(self, active: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ProgressTracker.QuorumActive per group (tracker.go:215-225)."""
        active = active if active is not None else self.active
        if active is None:
            raise ValueError("no RecentActive bits given")
        check_tensors(((active, "active", I16, self.G), (self.cfg, "cfg", I32, self.G)))
        out = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        _lib.call("qb_dev_csr_quorum_active", self.G, _ptr(self.cfg), _ptr(active), _ptr(out),
                  _stream(self.device))
        return out

    def tally_votes(self):
        """ProgressTracker.TallyVotes per group (tracker.go:267-288):
        (granted, rejected, VoteResult) as uint8 device tensors."""
        gr = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        rj = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        res = torch.empty(self.G, dtype=torch.uint8, device=self.device)
        _lib.call("qb_dev_csr_tally_votes", self.G, _ptr(self.cfg), _ptr(self.votes), _ptr(gr),
                  _ptr(rj), _ptr(res), _stream(self.device))
        return gr, rj, res

    def record_votes(self, batch: "AppRespBatch", group_term: torch.Tensor, prevote: bool = False,
                     stepdown_at: Optional[torch.Tensor] = None,
                     decided_at: Optional[torch.Tensor] = None,
                     stats: Optional[torch.Tensor] = None):
        """RecordVote for a batch of MsgVoteResp (or MsgPreVoteResp) records,
        first vote wins in batch order, polling stops at the group's VoteWon /
        VoteLost (tracker.go:258-288, raft.go:847-921, 1391-1414).
        Returns (stepdown_at, decided_at, stats)."""
        if stepdown_at is None:
            stepdown_at = torch.empty(self.G, dtype=torch.int32, device=self.device)
        if decided_at is None:
            decided_at = torch.empty(self.G, dtype=torch.int32, device=self.device)
        if stats is None:
            stats = torch.zeros(8, dtype=torch.int64, device=self.device)
        batch.check()
        check_tensors(((group_term, "group_term", I64, self.G),
                       (stepdown_at, "stepdown_at", I32, self.G),
                       (decided_at, "decided_at", I32, self.G),
                       (stats, "stats", I64, len(_lib.QB_VSTAT_NAMES))))
        need = _lib.load().qb_votes_workspace_bytes(batch.M)
        ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        _lib.call("qb_dev_record_votes", _lib.QB_VOTE_MODE_PREVOTE if prevote else
                  _lib.QB_VOTE_MODE_VOTE, self.G, batch.M, _ptr(batch.group), _ptr(batch.flags),
                  _ptr(batch.term), _ptr(group_term), _ptr(self.cfg), _ptr(self.votes),
                  _ptr(stepdown_at), _ptr(decided_at), _ptr(stats), _ptr(ws), ws.numel(),
                  _stream(self.device))
        return stepdown_at, decided_at, stats

    def validate(self, max_slots: Optional[int] = None) -> int:
        """Number of groups breaking the CSR invariants (off[0] == 0,
        0 <= s_g <= max_slots; default: this table's bound)."""
        bad = torch.zeros(1, dtype=torch.int64, device=self.device)
        ms = self.max_slots if max_slots is None else max_slots
        _lib.call("qb_dev_csr_validate", self.G, ms, _ptr(self.off), _ptr(bad),
                  _stream(self.device))
        return int(bad.item())


# -------------------------------------------------------------- tracker ---

@dataclass
class AppRespBatch:
    """A batch of MsgAppResp records (raftpb.Message fields the path reads)."""
    group: torch.Tensor  # int32 (uint32 group index)
    flags: torch.Tensor  # uint8: slot | 0x80 if Reject
    index: torch.Tensor  # int64 (uint64 Message.Index)
    term: torch.Tensor   # int64 (uint64 Message.Term)

    @property
    def M(self) -> int:
        return self.group.numel()

    def check(self) -> None:
        """Every column a contiguous device tensor of its dtype with M entries."""
        M = self.M
        check_tensors(((self.group, "batch.group", I32, 0), (self.flags, "batch.flags", U8, M),
                       (self.index, "batch.index", I64, M), (self.term, "batch.term", I64, M)))

    @classmethod
    def from_numpy(cls, group, slot, index, term, reject=None, device="cuda"):
        dev = torch.device(device)
        flags = np.asarray(slot, np.uint8) & 0x0F
        if reject is not None:
            flags = flags | (np.asarray(reject, bool).astype(np.uint8) << 7)
        return cls(torch.from_numpy(np.asarray(group, np.uint32).view(np.int32).copy()).to(dev),
                   torch.from_numpy(flags.astype(np.uint8)).to(dev),
                   from_u64(index, dev), from_u64(term, dev))


class FixedTracker:
    """Leader-side ProgressTracker state of G groups with n voters each."""

    def __init__(self, n: int, G: int, device="cuda", track_next: bool = False):
        self.n, self.G, self.device = n, G, torch.device(device)
        dev = self.device
        self.match = torch.zeros((n, G), dtype=torch.int64, device=dev)
        self.next = torch.ones((n, G), dtype=torch.int64, device=dev) if track_next else None
        self.active = torch.zeros(G + (G & 1), dtype=torch.int16, device=dev)  # even length
        self.term = torch.zeros(G, dtype=torch.int64, device=dev)
        self.term_start = torch.full((G,), -1, dtype=torch.int64, device=dev)  # ∞
        self.committed = torch.zeros(G, dtype=torch.int64, device=dev)
        self.stepdown_at = torch.full((G,), -1, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(_lib.QB_STAT_COUNT, dtype=torch.int64, device=dev)

    def apply_appresp(self, batch: AppRespBatch, reset_stats: bool = True):
        """stepLeader's MsgAppResp handling (quorum part) for a whole batch."""
        batch.check()
        if reset_stats:
            self.stats.zero_()
        _lib.call("qb_dev_fixed_apply_appresp", self.n, self.G, batch.M, _ptr(batch.group),
                  _ptr(batch.flags), _ptr(batch.index), _ptr(batch.term), _ptr(self.term),
                  _ptr(self.match), _ptr(self.next), _ptr(self.active), _ptr(self.stepdown_at),
                  _ptr(self.stats), _stream(self.device))

    def commit_advance(self, advanced_out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """raft.maybeCommit for every group; returns the per-group advanced flags."""
        check_tensors(((advanced_out, "advanced_out", FLAG, self.G),))
        _lib.call("qb_dev_fixed_commit_advance", self.n, self.G, _ptr(self.match),
                  _ptr(self.term_start), _ptr(self.committed), _ptr(advanced_out),
                  _stream(self.device))
        return advanced_out

    def step(self, batch: AppRespBatch, advanced_out: Optional[torch.Tensor] = None,
             reset_stats: bool = True, rearm: bool = True) -> Optional[torch.Tensor]:
        """One leader tick: apply the batch and run maybeCommit for every group
        (qb_dev_fixed_tracker_step: records bucketed by group, LDS atomics).

        The C step requires ``stepdown_at`` to hold UINT32_MAX on entry and
        writes it only for chunks holding a higher-term record
        (include/quorum_batch.h).  ``rearm=True`` (default) refills it first,
        so ``stepped_down()`` always describes this batch alone, as after
        ``apply_appresp``; ``rearm=False`` is the Go caller's protocol (it
        re-arms only the groups it stepped down; no per-group write per tick)."""
        batch.check()
        check_tensors(((advanced_out, "advanced_out", FLAG, self.G),))
        if reset_stats:
            self.stats.zero_()
        if rearm:
            self.stepdown_at.fill_(-1)
        need = _lib.load().qb_fixed_tracker_workspace_bytes(self.n, self.G, batch.M)
        if getattr(self, "_ws", None) is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        _lib.call("qb_dev_fixed_tracker_step", self.n, self.G, batch.M, _ptr(batch.group),
                  _ptr(batch.flags), _ptr(batch.index), _ptr(batch.term), _ptr(self.term),
                  _ptr(self.term_start), _ptr(self.match), _ptr(self.next), _ptr(self.active),
                  _ptr(self.committed), _ptr(self.stepdown_at), _ptr(advanced_out),
                  _ptr(self.stats), _ptr(self._ws), self._ws.numel(), _stream(self.device))
        return advanced_out

    def workspace(self, M: int) -> torch.Tensor:
        """A device workspace for one batch of M records (bucket / apply_bucketed)."""
        need = _lib.load().qb_fixed_tracker_workspace_bytes(self.n, self.G, M)
        return torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)

    def bucket(self, batch: AppRespBatch, ws: torch.Tensor, stream=None):
        """First half of ``step`` (qb_dev_fixed_tracker_bucket): the batch sorted
        by group into ``ws``; touches no tracker state, so it may run on another
        stream while the previous batch is applied."""
        batch.check()
        check_tensors(((ws, "ws", U8, 1),))
        _lib.call("qb_dev_fixed_tracker_bucket", self.n, self.G, batch.M, _ptr(batch.group),
                  _ptr(batch.flags), _ptr(batch.index), _ptr(batch.term), _ptr(ws), ws.numel(),
                  _stream(self.device) if stream is None else stream.cuda_stream)

    def apply_bucketed(self, batch: AppRespBatch, ws: torch.Tensor,
                       advanced_out: Optional[torch.Tensor] = None, stream=None):
        """Second half of ``step`` (qb_dev_fixed_tracker_apply) over a workspace
        that ``bucket`` filled for the same batch."""
        batch.check()
        check_tensors(((ws, "ws", U8, 1), (advanced_out, "advanced_out", FLAG, self.G)))
        _lib.call("qb_dev_fixed_tracker_apply", self.n, self.G, batch.M, _ptr(batch.group),
                  _ptr(batch.flags), _ptr(batch.index), _ptr(batch.term), _ptr(self.term),
                  _ptr(self.term_start), _ptr(self.match), _ptr(self.next), _ptr(self.active),
                  _ptr(self.committed), _ptr(self.stepdown_at), _ptr(advanced_out),
                  _ptr(self.stats), _ptr(ws), ws.numel(),
                  _stream(self.device) if stream is None else stream.cuda_stream)
        return advanced_out

    def stats_dict(self) -> dict:
        v = self.stats.cpu().tolist()
        return {k: v[i] for i, k in enumerate(_lib.QB_STAT_NAMES)}

    def stepped_down(self) -> torch.Tensor:
        """Groups whose leader stepped down in the last batch (a higher-term
        response, raft.go:875-879).  After ``step(..., rearm=False)`` a marker
        from an earlier batch stays until the caller re-arms that group."""
        return self.stepdown_at != -1

    def check_armed(self) -> None:
        """Opt-in check of the bucketed step's entry rule (every stepdown_at
        entry UINT32_MAX): qb_dev_stepdown_check_armed, synchronising."""
        scratch = torch.empty(1, dtype=torch.int64, device=self.device)
        _lib.call("qb_dev_stepdown_check_armed", self.G, _ptr(self.stepdown_at), _ptr(scratch),
                  _stream(self.device))


class CsrTracker:
    """Leader-side ProgressTracker state of G groups of the CSR layout (ragged
    voter counts, learners, joint configs): Progress.Match per slot, the
    leader's term, the first index of its term, the commit index and the
    RecentActive bits per group.  ``step`` = qb_dev_csr_tracker_step: a
    MsgAppResp batch applied and maybeCommit with the JointConfig
    CommittedIndex (tracker.go:162-179, joint.go:49-56, raft.go:585-588)."""

    def __init__(self, off: torch.Tensor, cfg: torch.Tensor, max_slots: Optional[int] = None,
                 device="cuda", track_next: bool = False):
        check_tensors(((off, "off", I32, cfg.numel() + 1), (cfg, "cfg", I32, 0)))
        self.off, self.cfg = off, cfg
        self.device = torch.device(device)
        self.G = cfg.numel()
        self.S = int(off[-1].item()) if self.G else 0
        if max_slots is None:
            max_slots = int((off[1:].long() - off[:-1].long()).max().item()) if self.G else 0
        self.max_slots = max(1, min(int(max_slots), _lib.QB_MAX_SLOTS))
        dev, G, S = self.device, self.G, max(self.S, 2)
        self.match = torch.zeros(S, dtype=torch.int64, device=dev)
        self.next = torch.ones(S, dtype=torch.int64, device=dev) if track_next else None
        self.active = torch.zeros(G + (G & 1), dtype=torch.int16, device=dev)
        self.term = torch.zeros(G, dtype=torch.int64, device=dev)
        self.term_start = torch.full((G,), -1, dtype=torch.int64, device=dev)  # ∞
        self.committed = torch.zeros(G, dtype=torch.int64, device=dev)
        self.stepdown_at = torch.full((G,), -1, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(_lib.QB_STAT_COUNT, dtype=torch.int64, device=dev)
        self._ws = None

    def committed_index(self) -> torch.Tensor:
        """ProgressTracker.Committed per group (JointConfig.CommittedIndex)."""
        c = torch.empty(self.G, dtype=torch.int64, device=self.device)
        _lib.call("qb_dev_csr_committed_vote", self.G, self.max_slots, _ptr(self.off),
                  _ptr(self.match), _ptr(self.cfg), None, _ptr(c), None, _stream(self.device))
        return c

    def commit_advance(self, advanced_out: Optional[torch.Tensor] = None):
        """maybeCommit for every group: the step with an empty batch."""
        empty = AppRespBatch(torch.zeros(1, dtype=torch.int32, device=self.device)[:0],
                             torch.zeros(1, dtype=torch.uint8, device=self.device)[:0],
                             torch.zeros(1, dtype=torch.int64, device=self.device)[:0],
                             torch.zeros(1, dtype=torch.int64, device=self.device)[:0])
        return self.step(empty, advanced_out, reset_stats=False)

    def step(self, batch: AppRespBatch, advanced_out: Optional[torch.Tensor] = None,
             reset_stats: bool = True, rearm: bool = True) -> Optional[torch.Tensor]:
        """One leader tick (qb_dev_csr_tracker_step); ``rearm`` as
        FixedTracker.step."""
        batch.check()
        check_tensors(((advanced_out, "advanced_out", FLAG, self.G),))
        if reset_stats:
            self.stats.zero_()
        if rearm:
            self.stepdown_at.fill_(-1)
        need = _lib.load().qb_csr_tracker_workspace_bytes(self.G, self.max_slots, batch.M)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        _lib.call("qb_dev_csr_tracker_step", self.G, self.max_slots, _ptr(self.off),
                  _ptr(self.cfg), batch.M, _ptr(batch.group), _ptr(batch.flags),
                  _ptr(batch.index), _ptr(batch.term), _ptr(self.term), _ptr(self.term_start),
                  _ptr(self.match), _ptr(self.next), _ptr(self.active), _ptr(self.committed),
                  _ptr(self.stepdown_at), _ptr(advanced_out), _ptr(self.stats), _ptr(self._ws),
                  self._ws.numel(), _stream(self.device))
        return advanced_out

    def stats_dict(self) -> dict:
        v = self.stats.cpu().tolist()
        return {k: v[i] for i, k in enumerate(_lib.QB_STAT_NAMES)}

    def stepped_down(self) -> torch.Tensor:
        """Groups whose leader stepped down in the last batch (a higher-term
        response, raft.go:875-879).  After ``step(..., rearm=False)`` a marker
        from an earlier batch stays until the caller re-arms that group."""
        return self.stepdown_at != -1

    def check_armed(self) -> None:
        """Opt-in check of the bucketed step's entry rule (every stepdown_at
        entry UINT32_MAX): qb_dev_stepdown_check_armed, synchronising."""
        scratch = torch.empty(1, dtype=torch.int64, device=self.device)
        _lib.call("qb_dev_stepdown_check_armed", self.G, _ptr(self.stepdown_at), _ptr(scratch),
                  _stream(self.device))
