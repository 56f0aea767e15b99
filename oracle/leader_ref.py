"""CPU restatement of etcd's leader inbox step — TEST INFRASTRUCTURE ONLY.

This module is a *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product package
(``etcd_amd``) never does.

It restates, one message at a time and in batch order, what a raft leader does
with the responses in its inbox.  Paths are relative
to the reference's ``raft/``:

  raft.Step term filter                        raft.go:847-921
  stepLeader, progress lookup                  raft.go:1099-1104
  MsgAppResp (reject: findConflictByTerm +     raft.go:1105-1283
    MaybeDecrTo; accept: MaybeUpdate, state
    transitions, maybeCommit, bcastAppend,
    maybeSendAppend loop, MsgTimeoutNow)
  MsgHeartbeatResp (+ ReadIndex acks)          raft.go:1284-1309
  MsgSnapStatus / MsgUnreachable               raft.go:1310-1342
  maybeSendAppend / sendAppend / bcastAppend   raft.go:423-492, 515-522
  maybeCommit                                  raft.go:585-588, log.go:328-334
  responseToReadIndexReq                       raft.go:1737-1752
  raftLog.term / entries / findConflictByTerm  log.go:268-299, 150-171
  Progress                                     tracker/progress.go:85-212
  Inflights                                    tracker/inflights.go:40-132
  readOnly.recvAck / advance                   read_only.go:68-121

Log model.  The step never appends, so the leader's raftLog is a static view:
``first`` (firstIndex; the dummy entry is first-1), ``last``, ``committed``,
the terms of [first-1, last] as runs ``[(start, term), ...]`` (ascending
starts, the first run starting at or before first-1), the storage snapshot
``(snap_index, snap_term)`` (snap_index 0 = ErrSnapshotTemporarilyUnavailable)
and ``max_ents``: how many entries ``raftLog.entries(lo, maxMsgSize)`` returns
(limitSize over entries of one size; at least one).

Pinning: tests/golden/leader_tables.json holds the reference's own table tests
for this path transcribed as data (progress_test.go, inflights_test.go, and the
raft_test.go scenarios TestLeaderAppResp, TestFastLogRejection,
TestProgressFlowControl, TestSendAppendForProgress*, TestHandleHeartbeatResp,
TestMsgAppRespWaitReset, TestRecvMsgUnreachable, TestRaftFreesReadOnlyMem);
tests/test_leader_oracle.py replays every one of them through this module.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

MAX_U64 = (1 << 64) - 1
M64 = MAX_U64

# tracker/state.go:26-33
STATE_PROBE, STATE_REPLICATE, STATE_SNAPSHOT = 0, 1, 2
STATE_NAMES = ("StateProbe", "StateReplicate", "StateSnapshot")

# raftpb/raft.pb.go:76-94 (MessageType), plus a local pseudo-type for a
# ReadState appended to raft.readStates (raft.go:1738-1743).
MSG_APP, MSG_APP_RESP, MSG_SNAP = 3, 4, 7
MSG_HEARTBEAT_RESP, MSG_UNREACHABLE, MSG_SNAP_STATUS = 9, 10, 11
MSG_TIMEOUT_NOW, MSG_READ_INDEX_RESP = 14, 16
READ_STATE = 255

# Inbound record kinds of the batch (the leader's inbox).
IN_APP_RESP, IN_HEARTBEAT_RESP, IN_SNAP_STATUS, IN_UNREACHABLE = 0, 1, 2, 3

READ_ONLY_SAFE, READ_ONLY_LEASE_BASED = 0, 1  # raft.go ReadOnlyOption

NO_SLOT = 0xFF  # raft.None as a slot


class Inflights:
    """tracker/inflights.go:22-132.  The buffer is allocated at full size; the
    reference grows it lazily, which never changes (start, count) or the FIFO
    contents, only buffer capacity."""

    def __init__(self, size: int, start: int = 0, count: int = 0, buffer=None):
        self.size = size
        self.start = start
        self.count = count
        self.buffer = list(buffer) if buffer is not None else [0] * size

    def clone(self):
        return Inflights(self.size, self.start, self.count, self.buffer)

    def add(self, inflight: int) -> None:
        """inflights.go:55-70."""
        if self.full():
            raise AssertionError("cannot add into a Full inflights")
        nxt = self.start + self.count
        if nxt >= self.size:
            nxt -= self.size
        self.buffer[nxt] = inflight
        self.count += 1

    def free_le(self, to: int) -> None:
        """inflights.go:88-116."""
        if self.count == 0 or to < self.buffer[self.start]:
            return
        idx = self.start
        i = 0
        while i < self.count:
            if to < self.buffer[idx]:
                break
            idx += 1
            if idx >= self.size:
                idx -= self.size
            i += 1
        self.count -= i
        self.start = idx
        if self.count == 0:
            self.start = 0

    def free_first_one(self) -> None:
        """inflights.go:118-120."""
        self.free_le(self.buffer[self.start])

    def full(self) -> bool:
        """inflights.go:122-125."""
        return self.count == self.size

    def reset(self) -> None:
        """inflights.go:128-132."""
        self.count = 0
        self.start = 0

    def fifo(self) -> List[int]:
        return [self.buffer[(self.start + k) % self.size] for k in range(self.count)]


@dataclass
class Progress:
    """tracker/progress.go:30-83 (the fields the leader step reads/writes)."""
    match: int = 0
    next: int = 0
    state: int = STATE_PROBE
    pending_snapshot: int = 0
    recent_active: bool = False
    probe_sent: bool = False
    inflights: Inflights = field(default_factory=lambda: Inflights(256))
    is_learner: bool = False

    def reset_state(self, state: int) -> None:
        """progress.go:85-92."""
        self.probe_sent = False
        self.pending_snapshot = 0
        self.state = state
        self.inflights.reset()

    def probe_acked(self) -> None:
        """progress.go:113-115."""
        self.probe_sent = False

    def become_probe(self) -> None:
        """progress.go:117-131."""
        if self.state == STATE_SNAPSHOT:
            pending = self.pending_snapshot
            self.reset_state(STATE_PROBE)
            self.next = max((self.match + 1) & M64, (pending + 1) & M64)
        else:
            self.reset_state(STATE_PROBE)
            self.next = (self.match + 1) & M64

    def become_replicate(self) -> None:
        """progress.go:133-137."""
        self.reset_state(STATE_REPLICATE)
        self.next = (self.match + 1) & M64

    def become_snapshot(self, snapshoti: int) -> None:
        """progress.go:139-144."""
        self.reset_state(STATE_SNAPSHOT)
        self.pending_snapshot = snapshoti

    def maybe_update(self, n: int) -> bool:
        """progress.go:146-157."""
        updated = False
        if self.match < n:
            self.match = n
            updated = True
            self.probe_acked()
        self.next = max(self.next, (n + 1) & M64)
        return updated

    def optimistic_update(self, n: int) -> None:
        """progress.go:159-161."""
        self.next = (n + 1) & M64

    def maybe_decr_to(self, rejected: int, match_hint: int) -> bool:
        """progress.go:163-191."""
        if self.state == STATE_REPLICATE:
            if rejected <= self.match:
                return False
            self.next = (self.match + 1) & M64
            return True
        if ((self.next - 1) & M64) != rejected:
            return False
        self.next = max(min(rejected, (match_hint + 1) & M64), 1)
        self.probe_sent = False
        return True

    def is_paused(self) -> bool:
        """progress.go:193-212."""
        if self.state == STATE_PROBE:
            return self.probe_sent
        if self.state == STATE_REPLICATE:
            return self.inflights.full()
        if self.state == STATE_SNAPSHOT:
            return True
        raise AssertionError("unexpected state")


@dataclass
class LogView:
    """The leader's raftLog as a batch of responses sees it (never appended
    to during the step).  runs: [(start_index, term)] covering [first-1, last]."""
    first: int
    last: int
    committed: int
    runs: list
    snap_index: int = 0
    snap_term: int = 0
    max_ents: int = 1 << 62

    def term(self, i: int) -> int:
        """log.go:268-288 (+ zeroTermOnErrCompacted): the valid range is
        [dummy, last]; anything outside has term 0."""
        dummy = self.first - 1
        if i < dummy or i > self.last:
            return 0
        t = 0
        for start, rt in self.runs:
            if start <= i:
                t = rt
        return t

    def entries(self, lo: int):
        """log.go:290-299 -> slice/mustCheckOutOfBounds (log.go:338-398):
        returns (n_entries, compacted)."""
        if lo > self.last:
            return 0, False
        if lo < self.first:
            return 0, True  # ErrCompacted
        return min(self.max_ents, self.last - lo + 1), False

    def find_conflict_by_term(self, index: int, term: int) -> int:
        """log.go:150-171."""
        if index > self.last:
            return index
        while True:
            if self.term(index) <= term:
                break
            index = (index - 1) & M64
        return index

    def maybe_commit(self, max_index: int, term: int) -> bool:
        """log.go:328-334 (+ commitTo, log.go:236-244)."""
        if max_index > self.committed and self.term(max_index) == term:
            self.committed = max_index
            return True
        return False


@dataclass
class ReadIndexStatus:
    """read_only.go:30-40: one pending read (ctx != 0; 0 is an empty context)."""
    ctx: int
    index: int
    acks: set
    from_slot: int  # NO_SLOT or the leader's slot -> local ReadState


@dataclass
class Msg:
    """An outbound message/event in the order the reference emits it."""
    type: int
    to: int
    index: int = 0
    log_term: int = 0
    commit: int = 0
    aux: int = 0  # MsgApp: number of entries; ReadIndexResp/ReadState: ctx

    def key(self):
        return (self.type, self.to, self.index, self.log_term, self.commit, self.aux)


@dataclass
class Inbound:
    kind: int
    slot: int
    term: int = 0
    index: int = 0     # MsgAppResp.Index; MsgHeartbeatResp: Context (0 = empty)
    reject: bool = False
    hint: int = 0      # RejectHint
    log_term: int = 0  # LogTerm (of the rejection hint)


class LeaderGroup:
    """One raft group whose node is the leader: Progress per slot (slot j is
    the j-th smallest ID; voters_in / voters_out as slot masks, learners are
    slots in neither), the log view, and the readOnly queue."""

    def __init__(self, n_slots: int, mask_in: int, mask_out: int, term: int, leader_slot: int,
                 log: LogView, progress: List[Progress], transferee: int = NO_SLOT,
                 read_only: int = READ_ONLY_SAFE, readq: Optional[List[ReadIndexStatus]] = None,
                 pending_readindex: bool = False):
        self.n_slots = n_slots
        self.mask_in, self.mask_out = mask_in, mask_out
        self.term = term
        self.leader_slot = leader_slot
        self.log = log
        self.prs = progress
        self.transferee = transferee
        self.read_only = read_only
        self.readq = readq if readq is not None else []
        self.pending_readindex = pending_readindex
        self.msgs: List[Msg] = []
        self.stepped_down_at: Optional[int] = None
        self.advanced = False
        self.released_pending = False

    def progress_string(self, slot: int) -> str:
        """Progress.String (tracker/progress.go:214-238); a slot in neither
        voter mask is a learner."""
        pr = self.prs[slot]
        out = f"{STATE_NAMES[pr.state]} match={pr.match} next={pr.next}"
        if not (((self.mask_in | self.mask_out) >> slot) & 1):
            out += " learner"
        if pr.is_paused():
            out += " paused"
        if pr.pending_snapshot > 0:
            out += f" pendingSnap={pr.pending_snapshot}"
        if not pr.recent_active:
            out += " inactive"
        n = pr.inflights.count
        if n > 0:
            out += f" inflight={n}"
            if pr.inflights.full():
                out += "[full]"
        return out

    # ----------------------------------------------------------- quorum ---
    def _voters(self, mask):
        return [s for s in range(self.n_slots) if (mask >> s) & 1]

    def committed_index(self) -> int:
        """tracker.go:177-179 -> joint.go:49-56 -> majority.go:126-172."""
        def ci(mask):
            vs = self._voters(mask)
            if not vs:
                return MAX_U64
            srt = sorted(self.prs[s].match for s in vs)
            return srt[len(vs) - (len(vs) // 2 + 1)]
        return min(ci(self.mask_in), ci(self.mask_out))

    def vote_result(self, acks: Optional[set]) -> int:
        """joint.go:61-75 over majority.go:178-210 with votes = acks (all
        true; None = a nil map)."""
        def vr(mask):
            vs = self._voters(mask)
            if not vs:
                return 3
            yes = sum(1 for s in vs if acks is not None and s in acks)
            missing = len(vs) - yes
            q = len(vs) // 2 + 1
            if yes >= q:
                return 3
            if yes + missing >= q:
                return 1
            return 2
        r1, r2 = vr(self.mask_in), vr(self.mask_out)
        if r1 == r2:
            return r1
        if r1 == 2 or r2 == 2:
            return 2
        return 1

    # ------------------------------------------------------------- send ---
    def maybe_send_append(self, to: int, send_if_empty: bool) -> bool:
        """raft.go:432-492."""
        pr = self.prs[to]
        if pr.is_paused():
            return False
        term = self.log.term((pr.next - 1) & M64)  # errt never set (log.go:268-288)
        n, compacted = self.log.entries(pr.next)
        if n == 0 and not send_if_empty:
            return False
        if compacted:
            if not pr.recent_active:
                return False
            if self.log.snap_index == 0:  # ErrSnapshotTemporarilyUnavailable
                return False
            self.msgs.append(Msg(MSG_SNAP, to, self.log.snap_index, self.log.snap_term, 0, 0))
            pr.become_snapshot(self.log.snap_index)
            return True
        m = Msg(MSG_APP, to, (pr.next - 1) & M64, term, self.log.committed, n)
        if n != 0:
            if pr.state == STATE_REPLICATE:
                last = (pr.next + n - 1) & M64
                pr.optimistic_update(last)
                pr.inflights.add(last)
            elif pr.state == STATE_PROBE:
                pr.probe_sent = True
            else:
                raise AssertionError("sending append in unhandled state")
        self.msgs.append(m)
        return True

    def send_append(self, to: int) -> None:
        """raft.go:423-425."""
        self.maybe_send_append(to, True)

    def bcast_append(self) -> None:
        """raft.go:515-522 (Visit goes in ascending ID = slot order)."""
        for s in range(self.n_slots):
            if s == self.leader_slot:
                continue
            self.send_append(s)

    def maybe_commit(self) -> bool:
        """raft.go:585-588."""
        return self.log.maybe_commit(self.committed_index(), self.term)

    def response_to_read_index_req(self, rs: ReadIndexStatus) -> None:
        """raft.go:1737-1752."""
        if rs.from_slot == NO_SLOT or rs.from_slot == self.leader_slot:
            self.msgs.append(Msg(READ_STATE, NO_SLOT, rs.index, 0, 0, rs.ctx))
        else:
            self.msgs.append(Msg(MSG_READ_INDEX_RESP, rs.from_slot, rs.index, 0, 0, rs.ctx))

    def propose(self, n: int) -> None:
        """Host-side op used only to replay the reference's scenarios between
        inbound batches: stepLeader MsgProp (raft.go:1019-1078) ->
        appendEntry (raft.go:621-642) -> bcastAppend."""
        li = self.log.last
        if self.log.runs[-1][1] != self.term:
            self.log.runs.append((li + 1, self.term))
        self.log.last = li + n
        self.prs[self.leader_slot].maybe_update(self.log.last)
        self.maybe_commit()
        self.bcast_append()

    # ------------------------------------------------------------- step ---
    def step(self, m: Inbound, batch_index: int = 0) -> str:
        """raft.Step's term filter (raft.go:847-921) then stepLeader.  Returns
        the class of the record: 'applied', 'stale', 'higher', 'nonmember',
        'after'."""
        if self.stepped_down_at is not None:
            return "after"
        if m.term == 0:
            pass  # local message (raft.go:849-850)
        elif m.term > self.term:
            # raft.go:852-880: a response from a higher term -> becomeFollower.
            self.stepped_down_at = batch_index
            return "higher"
        elif m.term < self.term:
            return "stale"  # raft.go:883-921: ignored
        if m.slot >= self.n_slots:
            return "nonmember"  # raft.go:1099-1104
        pr = self.prs[m.slot]
        if m.kind == IN_APP_RESP:
            self._app_resp(m, pr)
        elif m.kind == IN_HEARTBEAT_RESP:
            self._heartbeat_resp(m, pr)
        elif m.kind == IN_SNAP_STATUS:
            self._snap_status(m, pr)
        elif m.kind == IN_UNREACHABLE:
            # raft.go:1333-1338
            if pr.state == STATE_REPLICATE:
                pr.become_probe()
        return "applied"

    def _app_resp(self, m: Inbound, pr: Progress) -> None:
        """raft.go:1105-1283."""
        pr.recent_active = True
        if m.reject:
            next_probe = m.hint
            if m.log_term > 0:
                next_probe = self.log.find_conflict_by_term(m.hint, m.log_term)
            if pr.maybe_decr_to(m.index, next_probe):
                if pr.state == STATE_REPLICATE:
                    pr.become_probe()
                self.send_append(m.slot)
            return
        old_paused = pr.is_paused()
        if not pr.maybe_update(m.index):
            return
        if pr.state == STATE_PROBE:
            pr.become_replicate()
        elif pr.state == STATE_SNAPSHOT and pr.match >= pr.pending_snapshot:
            pr.become_probe()
            pr.become_replicate()
        elif pr.state == STATE_REPLICATE:
            pr.inflights.free_le(m.index)
        if self.maybe_commit():
            self.advanced = True
            if self.pending_readindex:
                # releasePendingReadIndexMessages (raft.go:1813-1825) runs on
                # the host: the engine reports it.
                self.pending_readindex = False
                self.released_pending = True
            self.bcast_append()
        elif old_paused:
            self.send_append(m.slot)
        while self.maybe_send_append(m.slot, False):
            pass
        if m.slot == self.transferee and pr.match == self.log.last:
            self.msgs.append(Msg(MSG_TIMEOUT_NOW, m.slot))

    def _heartbeat_resp(self, m: Inbound, pr: Progress) -> None:
        """raft.go:1284-1309."""
        pr.recent_active = True
        pr.probe_sent = False
        if pr.state == STATE_REPLICATE and pr.inflights.full():
            pr.inflights.free_first_one()
        if pr.match < self.log.last:
            self.send_append(m.slot)
        if self.read_only != READ_ONLY_SAFE or m.index == 0:
            return
        # read_only.go:68-79 recvAck
        acks = None
        for rs in self.readq:
            if rs.ctx == m.index:
                rs.acks.add(m.slot)
                acks = rs.acks
                break
        if self.vote_result(acks) != 3:
            return
        # read_only.go:84-121 advance
        for i, rs in enumerate(self.readq):
            if rs.ctx == m.index:
                released = self.readq[: i + 1]
                self.readq = self.readq[i + 1:]
                for r in released:
                    self.response_to_read_index_req(r)
                return

    def _snap_status(self, m: Inbound, pr: Progress) -> None:
        """raft.go:1310-1332."""
        if pr.state != STATE_SNAPSHOT:
            return
        if not m.reject:
            pr.become_probe()
        else:
            pr.pending_snapshot = 0
            pr.become_probe()
        pr.probe_sent = True


def run_batch(groups: List[LeaderGroup], records) -> dict:
    """Apply records [(group, Inbound)] in batch order; returns the stat counts
    keyed like the engine's QB_LSTAT_* counters."""
    stats = {"applied": 0, "stale": 0, "higher": 0, "nonmember": 0, "after": 0, "bad": 0}
    for i, (g, m) in enumerate(records):
        if g >= len(groups):
            stats["bad"] += 1
            continue
        stats[groups[g].step(m, i)] += 1
    return stats
