"""raft/quorum — the reference's API surface, backed by the batch engine.

``MajorityConfig``, ``JointConfig``, ``AckedIndexer`` and ``VoteResult`` keep
the Go package's names and semantics (quorum/quorum.go, majority.go,
joint.go).  ``CommittedIndex`` / ``VoteResult`` are computed by the HIP
kernels (one launch per call, or one launch for a whole list via
``committed_indexes`` / ``vote_results``); ``String``, ``Slice``,
``Describe`` and ``IDs`` are host-side formatting/set helpers, as in the
reference.  There is no CPU evaluation path.
"""
from __future__ import annotations

import enum
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch

from . import batch
from .batch import INDEX_INF

MAX_UINT64 = INDEX_INF


def index_string(i: int) -> str:
    """Index.String (quorum.go:25-30)."""
    return "∞" if i == MAX_UINT64 else str(i)


class VoteResult(enum.IntEnum):
    """quorum.VoteResult (quorum.go:45-58)."""
    VotePending = 1
    VoteLost = 2
    VoteWon = 3

    def __str__(self) -> str:  # voteresult_string.go:20-26
        return self.name


VotePending, VoteLost, VoteWon = VoteResult.VotePending, VoteResult.VoteLost, VoteResult.VoteWon


class AckedIndexer:
    """quorum.AckedIndexer (quorum.go:34-36)."""

    def AckedIndex(self, voter_id: int) -> Tuple[int, bool]:  # noqa: N802 (Go name)
        raise NotImplementedError


class MapAckIndexer(AckedIndexer, dict):
    """mapAckIndexer (quorum.go:38-43)."""

    def AckedIndex(self, voter_id: int) -> Tuple[int, bool]:  # noqa: N802
        if voter_id in self:
            return self[voter_id], True
        return 0, False


def _device(device) -> torch.device:
    if device is not None:
        return torch.device(device)
    return torch.device("cuda", torch.cuda.current_device())


class MajorityConfig(frozenset):
    """quorum.MajorityConfig: a set of voter IDs (majority.go:25)."""

    def String(self) -> str:  # noqa: N802
        return "(" + " ".join(str(i) for i in sorted(self)) + ")"

    __str__ = String

    def Slice(self) -> List[int]:  # noqa: N802
        return sorted(self)

    def Describe(self, l: AckedIndexer) -> str:  # noqa: N802, E741
        """majority.go:46-104 (debug text; host-side)."""
        if len(self) == 0:
            return "<empty majority quorum>"
        n = len(self)
        info = []
        for vid in self:
            idx, ok = l.AckedIndex(vid)
            info.append([vid, idx, ok, 0])
        info.sort(key=lambda t: (t[1], t[0]))
        for i in range(1, len(info)):
            if info[i - 1][1] < info[i][1]:
                info[i][3] = i
        info.sort(key=lambda t: t[0])
        out = [" " * n + "    idx\n"]
        for vid, idx, ok, bar in info:
            out.append(("?" + " " * n) if not ok else ("x" * bar + ">" + " " * (n - bar)))
            out.append(" %5d    (id=%d)\n" % (idx, vid))
        return "".join(out)

    def CommittedIndex(self, l: AckedIndexer, device=None) -> int:  # noqa: N802, E741
        return committed_indexes([JointConfig(self, MajorityConfig())], [l], device)[0]

    def VoteResult(self, votes: Mapping[int, bool], device=None) -> VoteResult:  # noqa: N802
        return vote_results([JointConfig(self, MajorityConfig())], [votes], device)[0]


class JointConfig(tuple):
    """quorum.JointConfig: [2]MajorityConfig (joint.go:19)."""

    def __new__(cls, c0: Iterable[int] = (), c1: Iterable[int] = ()):
        return super().__new__(cls, (MajorityConfig(c0), MajorityConfig(c1)))

    def String(self) -> str:  # noqa: N802  (joint.go:21-26)
        if len(self[1]) > 0:
            return self[0].String() + "&&" + self[1].String()
        return self[0].String()

    __str__ = String

    def IDs(self) -> set:  # noqa: N802  (joint.go:30-38)
        return set(self[0]) | set(self[1])

    def Describe(self, l: AckedIndexer) -> str:  # noqa: N802, E741  (joint.go:42-44)
        return MajorityConfig(self.IDs()).Describe(l)

    def CommittedIndex(self, l: AckedIndexer, device=None) -> int:  # noqa: N802, E741
        return committed_indexes([self], [l], device)[0]

    def VoteResult(self, votes: Mapping[int, bool], device=None) -> VoteResult:  # noqa: N802
        return vote_results([self], [votes], device)[0]


def _compile(configs: Sequence[JointConfig]) -> batch.CompiledConfigs:
    return batch.compile_configs([c[0] for c in configs], [c[1] for c in configs])


def committed_indexes(configs: Sequence[JointConfig], ackers: Sequence[AckedIndexer],
                      device=None) -> List[int]:
    """JointConfig.CommittedIndex for a list of groups in ONE kernel launch.

    A voter the AckedIndexer does not know counts as 0 (majority.go:149-161)."""
    if len(configs) != len(ackers):
        raise ValueError("one AckedIndexer per config")
    cc = _compile(configs)
    vals = np.zeros(len(cc.slot_ids), dtype=np.uint64)
    for g, l in enumerate(ackers):
        lo = int(cc.off[g])
        for j, vid in enumerate(cc.slots(g)):
            idx, ok = l.AckedIndex(int(vid))
            if ok:
                vals[lo + j] = idx
    grp = batch.CsrGroups.from_compiled(cc, vals, device=_device(device))
    out = grp.committed_index()
    return [int(x) for x in batch.as_u64(out)]


def vote_results(configs: Sequence[JointConfig], votes: Sequence[Mapping[int, bool]],
                 device=None) -> List[VoteResult]:
    """JointConfig.VoteResult for a list of groups in ONE kernel launch."""
    if len(configs) != len(votes):
        raise ValueError("one votes map per config")
    cc = _compile(configs)
    words = np.zeros(len(configs), dtype=np.uint32)
    for g, vm in enumerate(votes):
        vd = gr = 0
        for j, vid in enumerate(cc.slots(g)):
            vid = int(vid)
            if vid in vm:
                vd |= 1 << j
                if vm[vid]:
                    gr |= 1 << j
        words[g] = vd | (gr << 16)
    grp = batch.CsrGroups.from_compiled(cc, np.zeros(0, np.uint64), votes_u32=words,
                                        device=_device(device))
    out = grp.vote_result().cpu().numpy()
    return [VoteResult(int(x)) for x in out]


__all__ = ["AckedIndexer", "INDEX_INF", "JointConfig", "MAX_UINT64", "MajorityConfig",
           "MapAckIndexer", "VoteLost", "VotePending", "VoteResult", "VoteWon", "batch",
           "committed_indexes", "index_string", "vote_results"]
