"""etcd_amd — MI355X-native batched quorum engine for etcd's raft hot path.

Scope (BASELINE.json north_star): raft/quorum CommittedIndex /
VoteResult (majority and joint), the quorum-facing part of raft/tracker
(MsgAppResp MaybeUpdate scatter-max, commit advance with the term gate,
QuorumActive, RecordVote / TallyVotes), and the §8f rows around it: the
leader's full inbox step (Progress / Inflights / ReadIndex,
``etcd_amd.quorum.leader``), raftpb wire ingest (``etcd_amd.quorum.wire``)
and batched conf changes (``etcd_amd.quorum.confchange``) — evaluated for
millions of independent raft groups at once on HIP kernels (etcd_amd/csrc)
behind the C ABI in include/quorum_batch.h; ``etcd_amd.shard`` shards groups
over the GPUs of a node.
"""
from ._lib import QuorumBatchError, load  # noqa: F401

__version__ = "0.1.0"
