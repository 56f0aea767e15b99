"""CPU restatement of raft/confchange — TEST INFRASTRUCTURE ONLY.

Checker for the batched config-compile kernel.  Only
tests/ import it.  Paths relative to the reference's raft/:

  Changer.EnterJoint / LeaveJoint / Simple   confchange/confchange.go:49-152
  apply / makeVoter / makeLearner / remove   confchange/confchange.go:154-256
  initProgress                               confchange/confchange.go:258-281
  checkInvariants                            confchange/confchange.go:283-334
  symdiff / joint / nilAware*                confchange/confchange.go:358-410
  toConfChangeSingle / Restore               confchange/restore.go:26-155
  Config.String / Progress.String            tracker/tracker.go:80-93,
                                             tracker/progress.go:214-238,
                                             quorum/joint.go:21-26,
                                             quorum/majority.go:27-44

Sets use Python set / None exactly where the Go code keeps a map / nil.
Pinned by the reference's datadriven testdata (confchange/testdata/*.txt,
transcribed into tests/golden/confchange_datadriven.json) — see
tests/test_confchange_oracle.py.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass
from typing import Dict, Optional, Set

ADD_NODE, REMOVE_NODE, UPDATE_NODE, ADD_LEARNER = 0, 1, 2, 3  # raftpb ConfChangeType
TYPE_NAMES = {ADD_NODE: "ConfChangeAddNode", REMOVE_NODE: "ConfChangeRemoveNode",
              UPDATE_NODE: "ConfChangeUpdateNode", ADD_LEARNER: "ConfChangeAddLearnerNode"}


class ConfChangeError(Exception):
    pass


@dataclass
class Pr:
    """The Progress fields the Changer creates or carries (tracker/progress.go)."""
    match: int = 0
    next: int = 0
    state: int = 0
    probe_sent: bool = False
    pending_snapshot: int = 0
    recent_active: bool = False
    is_learner: bool = False
    inflight_count: int = 0
    inflight_size: int = 10
    tag: int = -1  # test-only identity of carried Progress

    def string(self) -> str:
        """progress.go:214-238."""
        s = f"{('StateProbe', 'StateReplicate', 'StateSnapshot')[self.state]} match={self.match} next={self.next}"
        if self.is_learner:
            s += " learner"
        paused = (self.probe_sent if self.state == 0 else
                  (self.inflight_count == self.inflight_size if self.state == 1 else True))
        if paused:
            s += " paused"
        if self.pending_snapshot > 0:
            s += f" pendingSnap={self.pending_snapshot}"
        if not self.recent_active:
            s += " inactive"
        if self.inflight_count > 0:
            s += f" inflight={self.inflight_count}"
            if self.inflight_count == self.inflight_size:
                s += "[full]"
        return s


@dataclass
class Tracker:
    voters_in: Set[int]
    voters_out: Optional[Set[int]]
    learners: Optional[Set[int]]
    learners_next: Optional[Set[int]]
    auto_leave: bool
    prs: Dict[int, Pr]
    max_inflight: int = 10

    @classmethod
    def empty(cls, max_inflight=10):
        """tracker.MakeProgressTracker (tracker.go:129-141)."""
        return cls(set(), None, None, None, False, {}, max_inflight)

    def config_string(self) -> str:
        """tracker.go:80-93 with JointConfig / MajorityConfig String."""
        def ms(s):
            return "(" + " ".join(str(x) for x in sorted(s)) + ")"
        v = ms(self.voters_in)
        if self.voters_out:
            v += "&&" + ms(self.voters_out)
        out = f"voters={v}"
        if self.learners is not None:
            out += f" learners={ms(self.learners)}"
        if self.learners_next is not None:
            out += f" learners_next={ms(self.learners_next)}"
        if self.auto_leave:
            out += " autoleave"
        return out

    def progress_string(self) -> str:
        """ProgressMap.String (progress.go:243-257)."""
        return "".join(f"{i}: {self.prs[i].string()}\n" for i in sorted(self.prs))


def _joint(t: Tracker) -> bool:
    return bool(t.voters_out)


def _nil_add(s, x):
    s = set() if s is None else s
    s.add(x)
    return s


def _nil_del(s, x):
    if s is None:
        return None
    s.discard(x)
    return s if s else None


def check_invariants(t: Tracker) -> None:
    """confchange.go:283-334 (the first violation in ascending ID order)."""
    ids = set(t.voters_in) | set(t.voters_out or ())
    for group in (sorted(ids), sorted(t.learners or ()), sorted(t.learners_next or ())):
        for i in group:
            if i not in t.prs:
                raise ConfChangeError(f"no progress for {i}")
    for i in sorted(t.learners_next or ()):
        if i not in (t.voters_out or ()):
            raise ConfChangeError(f"{i} is in LearnersNext, but not Voters[1]")
        if t.prs[i].is_learner:
            raise ConfChangeError(f"{i} is in LearnersNext, but is already marked as learner")
    for i in sorted(t.learners or ()):
        if i in (t.voters_out or ()):
            raise ConfChangeError(f"{i} is in Learners and Voters[1]")
        if i in t.voters_in:
            raise ConfChangeError(f"{i} is in Learners and Voters[0]")
        if not t.prs[i].is_learner:
            raise ConfChangeError(f"{i} is in Learners, but is not marked as learner")
    if not _joint(t):
        if t.voters_out is not None:
            raise ConfChangeError("cfg.Voters[1] must be nil when not joint")
        if t.learners_next is not None:
            raise ConfChangeError("cfg.LearnersNext must be nil when not joint")
        if t.auto_leave:
            raise ConfChangeError("AutoLeave must be false when not joint")


class Changer:
    """confchange.go:30-33."""

    def __init__(self, tracker: Tracker, last_index: int):
        self.t = tracker
        self.last_index = last_index

    def _copy(self) -> Tracker:
        """checkAndCopy (confchange.go:336-349)."""
        t = copy.deepcopy(self.t)
        check_invariants(t)
        return t

    def enter_joint(self, auto_leave: bool, ccs) -> Tracker:
        """confchange.go:49-76."""
        t = self._copy()
        if _joint(t):
            raise ConfChangeError("config is already joint")
        if len(t.voters_in) == 0:
            raise ConfChangeError("can't make a zero-voter config joint")
        t.voters_out = set(t.voters_in)
        self._apply(t, ccs)
        t.auto_leave = auto_leave
        check_invariants(t)
        return t

    def leave_joint(self) -> Tracker:
        """confchange.go:91-120."""
        t = self._copy()
        if not _joint(t):
            raise ConfChangeError("can't leave a non-joint config")
        for i in sorted(t.learners_next or ()):
            t.learners = _nil_add(t.learners, i)
            t.prs[i].is_learner = True
        t.learners_next = None
        for i in sorted(t.voters_out or ()):
            if i not in t.voters_in and i not in (t.learners or ()):
                del t.prs[i]
        t.voters_out = None
        t.auto_leave = False
        check_invariants(t)
        return t

    def simple(self, ccs) -> Tracker:
        """confchange.go:127-146."""
        t = self._copy()
        if _joint(t):
            raise ConfChangeError("can't apply simple config change in joint config")
        self._apply(t, ccs)
        if len(self.t.voters_in ^ t.voters_in) > 1:
            raise ConfChangeError("more than one voter changed without entering joint config")
        check_invariants(t)
        return t

    def _apply(self, t: Tracker, ccs) -> None:
        """confchange.go:151-175."""
        for typ, node in ccs:
            if node == 0:
                continue
            if typ == ADD_NODE:
                self._make_voter(t, node)
            elif typ == ADD_LEARNER:
                self._make_learner(t, node)
            elif typ == REMOVE_NODE:
                self._remove(t, node)
            elif typ == UPDATE_NODE:
                pass
            else:
                raise ConfChangeError(f"unexpected conf type {typ}")
        if len(t.voters_in) == 0:
            raise ConfChangeError("removed all voters")

    def _make_voter(self, t, i):
        """confchange.go:177-190."""
        pr = t.prs.get(i)
        if pr is None:
            self._init_progress(t, i, False)
            return
        pr.is_learner = False
        t.learners = _nil_del(t.learners, i)
        t.learners_next = _nil_del(t.learners_next, i)
        t.voters_in.add(i)

    def _make_learner(self, t, i):
        """confchange.go:204-227."""
        pr = t.prs.get(i)
        if pr is None:
            self._init_progress(t, i, True)
            return
        if pr.is_learner:
            return
        self._remove(t, i)
        t.prs[i] = pr
        if i in (t.voters_out or ()):
            t.learners_next = _nil_add(t.learners_next, i)
        else:
            pr.is_learner = True
            t.learners = _nil_add(t.learners, i)

    def _remove(self, t, i):
        """confchange.go:230-245."""
        if i not in t.prs:
            return
        t.voters_in.discard(i)
        t.learners = _nil_del(t.learners, i)
        t.learners_next = _nil_del(t.learners_next, i)
        if i not in (t.voters_out or ()):
            del t.prs[i]

    def _init_progress(self, t, i, is_learner):
        """confchange.go:258-281."""
        if not is_learner:
            t.voters_in.add(i)
        else:
            t.learners = _nil_add(t.learners, i)
        t.prs[i] = Pr(match=0, next=self.last_index, is_learner=is_learner, recent_active=True,
                      inflight_size=t.max_inflight)


def to_conf_change_single(voters, learners, voters_outgoing, learners_next):
    """restore.go:26-92."""
    out = [(ADD_NODE, i) for i in voters_outgoing]
    inc = [(REMOVE_NODE, i) for i in voters_outgoing]
    inc += [(ADD_NODE, i) for i in voters]
    inc += [(ADD_LEARNER, i) for i in learners]
    inc += [(ADD_LEARNER, i) for i in learners_next]
    return out, inc


def restore(tracker: Tracker, last_index: int, voters, learners, voters_outgoing, learners_next,
            auto_leave: bool) -> Tracker:
    """restore.go:116-155 (chain of Simple / EnterJoint)."""
    out, inc = to_conf_change_single(voters, learners, voters_outgoing, learners_next)
    t = tracker
    if not out:
        for cc in inc:
            t = Changer(t, last_index).simple([cc])
    else:
        for cc in out:
            t = Changer(t, last_index).simple([cc])
        t = Changer(t, last_index).enter_joint(auto_leave, inc)
    return t


def parse_ccs(text: str):
    """datadriven_test.go:47-75 tokens: vN, lN, rN, uN."""
    toks = text.strip().split(" ")
    if toks == [""]:
        return []
    out = []
    for tok in toks:
        typ = {"v": ADD_NODE, "l": ADD_LEARNER, "r": REMOVE_NODE, "u": UPDATE_NODE}[tok[0]]
        out.append((typ, int(tok[1:])))
    return out


def run_datadriven(cases) -> list:
    """datadriven_test.go:28-109: one tracker per file, LastIndex incremented
    after every command; returns the output text of every case."""
    t = Tracker.empty(10)
    last_index = 0
    outs = []
    for c in cases:
        ccs = parse_ccs(c["input"])
        try:
            ch = Changer(t, last_index)
            if c["cmd"] == "simple":
                nt = ch.simple(ccs)
            elif c["cmd"] == "enter-joint":
                nt = ch.enter_joint(c.get("autoleave", False), ccs)
            elif c["cmd"] == "leave-joint":
                if ccs:
                    raise ConfChangeError("this command takes no input")
                nt = ch.leave_joint()
            else:
                raise ConfChangeError("unknown command")
            t = nt
            outs.append(t.config_string() + "\n" + t.progress_string())
        except ConfChangeError as e:
            outs.append(str(e) + "\n")
        last_index += 1
    return outs
