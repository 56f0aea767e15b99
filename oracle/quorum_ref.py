"""CPU restatement of etcd's raft quorum/tracker hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product package
(``etcd_amd``) never does, and nothing here is ever the thing measured or
shipped.

Pinning: every function below is a line-by-line restatement of the reference Go
code cited in its docstring (paths relative to the reference's ``raft/``), and
the restatement is pinned by the reference's own known-answer data committed in
``tests/golden/`` (127 datadriven cases with their full Describe() output, plus
the TestCommit / TestLeaderElectionInOneRoundRPC / TestProgressUpdate tables),
see ``tests/test_oracle_golden.py``.  The reference (Go) cannot be built or run
in this image (no Go toolchain), so it is not used as a second oracle.

Pure-Python loops: use for small cases only.  The C restatement in
``oracle/quorum_oracle.c`` is the full-size checker and is itself validated
against this module.
"""
from __future__ import annotations

MAX_U64 = (1 << 64) - 1

# quorum.go:45-58 — VoteResult enum (1-based; 0 is not a valid result).
VOTE_PENDING = 1
VOTE_LOST = 2
VOTE_WON = 3
VOTE_NAMES = {VOTE_PENDING: "VotePending", VOTE_LOST: "VoteLost", VOTE_WON: "VoteWon"}


def index_string(i: int) -> str:
    """quorum.go:25-30 — Index.String(): MaxUint64 prints as the infinity sign."""
    return "∞" if i == MAX_U64 else str(i)


def vote_string(v: int) -> str:
    """voteresult_string.go:20-26."""
    return VOTE_NAMES.get(v, f"VoteResult({v})")


def insertion_sort(sl: list) -> None:
    """majority.go:115-122 — in-place ascending insertion sort."""
    a, b = 0, len(sl)
    for i in range(a + 1, b):
        j = i
        while j > a and sl[j] < sl[j - 1]:
            sl[j], sl[j - 1] = sl[j - 1], sl[j]
            j -= 1


def majority_committed_index(c, acked) -> int:
    """majority.go:126-172 — MajorityConfig.CommittedIndex.

    ``c`` is an iterable of voter IDs (a set), ``acked`` a mapping id -> index
    (the AckedIndexer; a missing key is ``found == false``).
    """
    c = list(c)
    n = len(c)
    if n == 0:
        return MAX_U64                                   # majority.go:128-133
    srt = [0] * n                                         # majority.go:141-147
    i = n - 1                                             # majority.go:149-161
    for vid in c:
        if vid in acked:
            srt[i] = acked[vid]
            i -= 1
    insertion_sort(srt)                                   # majority.go:165
    pos = n - (n // 2 + 1)                                # majority.go:170
    return srt[pos]


def majority_vote_result(c, votes) -> int:
    """majority.go:178-210 — MajorityConfig.VoteResult."""
    c = list(c)
    if len(c) == 0:
        return VOTE_WON                                   # majority.go:179-184
    no, yes, missing = 0, 0, 0
    for vid in c:                                         # majority.go:186-200
        if vid not in votes:
            missing += 1
            continue
        if votes[vid]:
            yes += 1
        else:
            no += 1
    q = len(c) // 2 + 1                                   # majority.go:202
    if yes >= q:
        return VOTE_WON
    if yes + missing >= q:
        return VOTE_PENDING
    return VOTE_LOST


def joint_committed_index(c0, c1, acked) -> int:
    """joint.go:49-56 — JointConfig.CommittedIndex: min of both halves."""
    i0 = majority_committed_index(c0, acked)
    i1 = majority_committed_index(c1, acked)
    return i0 if i0 < i1 else i1


def joint_vote_result(c0, c1, votes) -> int:
    """joint.go:61-75 — JointConfig.VoteResult."""
    r1 = majority_vote_result(c0, votes)
    r2 = majority_vote_result(c1, votes)
    if r1 == r2:
        return r1
    if r1 == VOTE_LOST or r2 == VOTE_LOST:
        return VOTE_LOST
    return VOTE_PENDING


def alternative_majority_committed_index(c, acked) -> int:
    """quick_test.go:85-122 — the "dumb" counting formulation."""
    c = list(c)
    if len(c) == 0:
        return MAX_U64
    id_to_idx = {vid: acked[vid] for vid in c if vid in acked}
    idx_to_votes = {idx: 0 for idx in id_to_idx.values()}
    for idx in id_to_idx.values():
        for idy in idx_to_votes:
            if idy > idx:
                continue
            idx_to_votes[idy] += 1
    q = len(c) // 2 + 1
    max_quorum_idx = 0
    for idx, n in idx_to_votes.items():
        if n >= q and idx > max_quorum_idx:
            max_quorum_idx = idx
    return max_quorum_idx


def majority_describe(c, acked) -> str:
    """majority.go:46-104 — MajorityConfig.Describe (host-side debug text)."""
    c = list(c)
    if len(c) == 0:
        return "<empty majority quorum>"
    n = len(c)
    info = []
    for vid in c:
        ok = vid in acked
        info.append({"id": vid, "idx": acked.get(vid, 0), "ok": ok, "bar": 0})
    info.sort(key=lambda t: (t["idx"], t["id"]))          # majority.go:73-78
    for i in range(len(info)):                            # majority.go:81-85
        if i > 0 and info[i - 1]["idx"] < info[i]["idx"]:
            info[i]["bar"] = i
    info.sort(key=lambda t: t["id"])                      # majority.go:88-90
    buf = [" " * n + "    idx\n"]
    for t in info:
        bar = t["bar"]
        if not t["ok"]:
            buf.append("?" + " " * n)
        else:
            buf.append("x" * bar + ">" + " " * (n - bar))
        buf.append(" %5d    (id=%d)\n" % (t["idx"], t["id"]))
    return "".join(buf)


def joint_ids(c0, c1):
    """joint.go:30-38 — JointConfig.IDs."""
    return set(c0) | set(c1)


# --------------------------------------------------------------------------
# tracker / log restatement
# --------------------------------------------------------------------------

def progress_maybe_update(match: int, nxt: int, n: int):
    """tracker/progress.go:144-153 — Progress.MaybeUpdate.

    Returns (match, next, updated).  ProbeSent bookkeeping (ProbeAcked) is
    flow-control state outside this path.
    """
    updated = False
    if match < n:
        match = n
        updated = True
    nxt = max(nxt, n + 1)
    return match, nxt, updated


def log_term(entries_term_of, i: int) -> int:
    """log.go:262-287 with zeroTermOnErrCompacted (log.go:400-406): an index
    outside the stored log has term 0."""
    return entries_term_of(i)


def log_maybe_commit(committed: int, max_index: int, term: int, term_of) -> int:
    """log.go:328-334 (+ commitTo log.go:236-244): returns the new committed."""
    if max_index > committed and term_of(max_index) == term:
        return max_index
    return committed


def window_term_of(term_start: int, last_index: int, term: int):
    """A leader's log restricted to what the gate can observe: entries
    [term_start, last_index] carry the leader's current ``term`` and every
    other index carries a different (older) term or is absent (term 0).
    This is exact for a leader because terms are non-decreasing along the log
    and the leader appended an entry of its own term at becomeLeader
    (raft.go:747-748)."""
    def term_of(i):
        if term_start <= i <= last_index:
            return term
        return -1 if 1 <= i <= last_index else 0
    return term_of


def tracker_tally_votes(voters_in, voters_out, learners, votes):
    """tracker.go:267-288 — ProgressTracker.TallyVotes; the progress map holds
    every voter and learner (confchange invariant)."""
    granted = rejected = 0
    for vid in joint_ids(voters_in, voters_out) | set(learners):
        if vid in learners:
            continue
        if vid not in votes:
            continue
        if votes[vid]:
            granted += 1
        else:
            rejected += 1
    return granted, rejected, joint_vote_result(voters_in, voters_out, votes)


def tracker_record_vote(votes: dict, vid: int, v: bool) -> None:
    """tracker.go:258-263 — first vote wins."""
    if vid not in votes:
        votes[vid] = v


def tracker_quorum_active(voters_in, voters_out, learners, recent_active: dict) -> bool:
    """tracker.go:215-225 — QuorumActive."""
    votes = {}
    for vid in sorted(joint_ids(voters_in, voters_out) | set(learners)):
        if vid in learners:
            continue
        votes[vid] = recent_active.get(vid, False)
    return joint_vote_result(voters_in, voters_out, votes) == VOTE_WON


# --------------------------------------------------------------------------
# The datadriven harness, restated (datadriven_test.go:36-250)
# --------------------------------------------------------------------------

def _make_lookuper(vals, ids, idsj):
    """datadriven_test.go:124-155 — placeholders (0) are removed afterwards."""
    l = {}
    p = 0
    for vid in list(ids) + list(idsj):
        if vid in l:
            continue
        if p < len(vals):
            l[vid] = vals[p]
            p += 1
    return {k: v for k, v in l.items() if v != 0}


def datadriven_output(case) -> str:
    """Run one datadriven case the way datadriven_test.go:36-250 does and
    return the text it would print (Describe output + result line)."""
    ids = case["cfg"]
    joint = case["cfgj"] is not None
    idsj = case["cfgj"] or []
    idxs = [0 if v is None else v for v in case["idx"]]
    votes = case["votes"]
    c = set(ids)
    cj = set(idsj)

    inp = votes if case["cmd"] == "vote" else idxs
    voters = joint_ids(c, cj)
    if len(voters) != len(inp):
        return "error: mismatched input (explicit or _) for voters %s: %s\n" % (voters, inp)

    buf = []
    if case["cmd"] == "committed":
        l = _make_lookuper(idxs, ids, idsj)
        if not joint:
            idx = majority_committed_index(c, l)
            buf.append(majority_describe(c, l))
            a = alternative_majority_committed_index(c, l)
            if a != idx:
                buf.append("%s <-- via alternative computation\n" % index_string(a))
            a = joint_committed_index(c, set(), l)
            if a != idx:
                buf.append("%s <-- via zero-joint quorum\n" % index_string(a))
            a = joint_committed_index(c, c, l)
            if a != idx:
                buf.append("%s <-- via self-joint quorum\n" % index_string(a))

            def overlay(cc, ll, oid, oidx):
                out = {}
                for iid in cc:
                    if iid == oid:
                        out[iid] = oidx
                    elif iid in ll:
                        out[iid] = ll[iid]
                return out

            for vid in c:
                iidx = l.get(vid, 0)
                if idx > iidx and iidx > 0:
                    lo = overlay(c, l, vid, iidx - 1)
                    a = majority_committed_index(c, lo)
                    if a != idx:
                        buf.append("%s <-- overlaying %d->%d" % (index_string(a), vid, iidx))
                    lo = overlay(c, l, vid, 0)
                    a = majority_committed_index(c, lo)
                    if a != idx:
                        buf.append("%s <-- overlaying %d->0" % (index_string(a), vid))
            buf.append("%s\n" % index_string(idx))
        else:
            buf.append(majority_describe(voters, l))
            idx = joint_committed_index(c, cj, l)
            a = joint_committed_index(cj, c, l)
            if a != idx:
                buf.append("%s <-- via symmetry\n" % index_string(a))
            buf.append("%s\n" % index_string(idx))
    elif case["cmd"] == "vote":
        ll = _make_lookuper(votes, ids, idsj)
        l = {k: v != 1 for k, v in ll.items()}
        if not joint:
            buf.append("%s\n" % vote_string(majority_vote_result(c, l)))
        else:
            r = joint_vote_result(c, cj, l)
            ar = joint_vote_result(cj, c, l)
            if ar != r:
                buf.append("%s <-- via symmetry\n" % vote_string(ar))
            buf.append("%s\n" % vote_string(r))
    else:
        raise ValueError(case["cmd"])
    return "".join(buf)


def datadriven_inputs(case):
    """(c0, c1, acked, votes) for one datadriven case, as the harness builds
    them (datadriven_test.go:111-155)."""
    ids = case["cfg"]
    idsj = case["cfgj"] or []
    idxs = [0 if v is None else v for v in case["idx"]]
    acked = _make_lookuper(idxs, ids, idsj)
    vl = _make_lookuper(case["votes"], ids, idsj)
    votes = {k: v != 1 for k, v in vl.items()}
    return set(ids), set(idsj), acked, votes


# --------------------------------------------------------------------------
# Vote responses, one record at a time (the sequential (pre-)candidate)
# --------------------------------------------------------------------------

STAT_RECORDED, STAT_DUPLICATE, STAT_STALE, STAT_HIGHER, STAT_AFTER, STAT_BAD = range(6)


STAT_AFTER_DECISION = 6


class Candidate:
    """The quorum-facing state of a (pre-)candidate taking its vote responses
    one at a time, in batch order (raft.go:847-921 Step's term handling,
    raft.go:1383-1414 stepCandidate, raft.go:837-845 poll, tracker.go:258-288
    RecordVote / TallyVotes).  ``votes`` maps slot -> granted; c0 / c1 are the
    slot sets of JointConfig halves Voters[0] / Voters[1].

    At VoteWon / VoteLost the node changes state (raft.go:1402-1414): a
    pre-candidate campaigns (becomeCandidate: term + 1, raft.go:1403), a
    candidate becomes leader, a loser becomes follower at its term.  None of
    them polls another response of this kind (a candidate's myVoteRespType is
    MsgVoteResp, raft.go:1385-1390; leaders and followers do not handle vote
    responses); a response above the node's current term still makes it
    becomeFollower — except a granted MsgPreVoteResp, which never changes the
    term (raft.go:866-871).  The new election's ResetVotes and self vote
    (campaign) are not modelled: the votes stay as they stood at the decision."""

    def __init__(self, prevote: bool, term: int, c0, c1, votes: dict):
        self.prevote, self.term = prevote, term
        self.c0, self.c1, self.votes = set(c0), set(c1), votes
        self.state = "PreCandidate" if prevote else "Candidate"
        self.down = False
        self.decided = False

    def step(self, slot: int, reject: bool, term: int) -> int:
        if self.down:
            return STAT_AFTER
        if term > self.term and not (self.prevote and not reject):
            self.term, self.state, self.down = term, "Follower", True  # becomeFollower
            return STAT_HIGHER
        mine = self.state == ("PreCandidate" if self.prevote else "Candidate")
        if not mine:
            return STAT_AFTER_DECISION
        if term < self.term:
            return STAT_STALE
        # poll -> RecordVote (first vote wins) -> TallyVotes
        stat = STAT_DUPLICATE if slot in self.votes else STAT_RECORDED
        self.votes.setdefault(slot, not reject)
        res = joint_vote_result(self.c0, self.c1, self.votes)
        if res == VOTE_WON:
            self.decided = True
            if self.prevote:
                self.term, self.state = self.term + 1, "Candidate"  # campaign(campaignElection)
            else:
                self.state = "Leader"
        elif res == VOTE_LOST:
            self.decided = True
            self.state = "Follower"
        return stat


def tally_votes_slots(mask_in: int, mask_out: int, votes: dict):
    """TallyVotes (tracker.go:267-288) on slot-indexed votes: (granted,
    rejected, JointConfig.VoteResult)."""
    voters = mask_in | mask_out
    granted = sum(1 for s, v in votes.items() if (voters >> s) & 1 and v)
    rejected = sum(1 for s, v in votes.items() if (voters >> s) & 1 and not v)
    c0 = {s for s in range(16) if (mask_in >> s) & 1}
    c1 = {s for s in range(16) if (mask_out >> s) & 1}
    return granted, rejected, joint_vote_result(c0, c1, votes)
