"""GPU parity for batched elections: RecordVote (first vote wins, batch
order, term filter for MsgVoteResp / MsgPreVoteResp, step-down ordering) and
TallyVotes, against the one-record-at-a-time oracle."""
import numpy as np
import pytest
import torch

from etcd_amd import quorum
from etcd_amd.quorum import VoteResult, batch
from oracle import quorum_ref as q
from tests import oracle_c as oc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(prevote, G, M, seed, p_dup=0.3):
    rng = np.random.default_rng(seed)
    grp = batch.CsrGroups.synth(0x5EED0007, "joint" if seed % 2 else "ragged", G, device=DEV)
    off = grp.off.cpu().numpy().view(np.uint32)
    cfg = grp.cfg.cpu().numpy().view(np.uint32)
    # pre-batch votes: a few slots already voted
    votes0 = np.zeros(G, np.uint32)
    pre = {}
    for g in range(G):
        s = int(off[g + 1] - off[g])
        d = {}
        for j in range(s):
            if rng.random() < 0.1:
                d[j] = bool(rng.random() < 0.5)
        pre[g] = d
        vd = sum(1 << j for j in d)
        gr = sum(1 << j for j, v in d.items() if v)
        votes0[g] = vd | (gr << 16)
    grp.votes.copy_(torch.from_numpy(votes0.view(np.int32)))
    gterm = rng.integers(3, 9, size=G).astype(np.uint64)
    group = rng.integers(0, G + 3, size=M).astype(np.uint32)  # a few bad groups
    sizes = np.diff(off.astype(np.int64))
    gg = np.minimum(group, G - 1)
    slot = (rng.integers(0, 1 << 30, size=M) % np.maximum(sizes[gg], 1)).astype(np.uint8)
    # duplicates: repeat earlier (group, slot) pairs, often with the opposite vote
    for i in range(1, M):
        if rng.random() < p_dup:
            j = rng.integers(0, i)
            group[i], slot[i] = group[j], slot[j]
    reject = rng.random(M) < 0.4
    dt = rng.choice([-1, 0, 0, 0, 0, 0, 1], size=M)
    term = np.where(group < G, gterm[gg].astype(np.int64) + dt, 5).astype(np.uint64)
    flags = (slot | (reject.astype(np.uint8) << 7)).astype(np.uint8)

    # oracle
    stats = np.zeros(6, np.int64)
    down = np.zeros(G, bool)
    first_down = np.full(G, 0xFFFFFFFF, np.uint32)
    for i in range(M):
        g = int(group[i])
        if g >= G:
            stats[q.STAT_BAD] += 1
            continue
        st, d = q.vote_response_sequential(prevote, int(gterm[g]), bool(down[g]), pre[g],
                                           int(slot[i]), bool(reject[i]), int(term[i]))
        if st == q.STAT_HIGHER and first_down[g] == 0xFFFFFFFF:
            first_down[g] = i
        down[g] = d
        stats[st] += 1

    b = batch.AppRespBatch.from_numpy(group, slot, np.zeros(M, np.uint64), term, reject,
                                      device=DEV)
    sd, gst = grp.record_votes(b, batch.from_u64(gterm, DEV), prevote=prevote)
    got_votes = grp.votes.cpu().numpy().view(np.uint32)
    for g in range(G):
        d = pre[g]
        vd = sum(1 << j for j in d)
        gr = sum(1 << j for j, v in d.items() if v)
        assert got_votes[g] == (vd | (gr << 16)), g
    assert np.array_equal(sd.cpu().numpy().view(np.uint32), first_down)
    assert gst.cpu().numpy()[:6].tolist() == stats.tolist()
    gr_, rj_, res = grp.tally_votes()
    gr_, rj_, res = gr_.cpu().numpy(), rj_.cpu().numpy(), res.cpu().numpy()
    for g in range(G):
        eg, er, eres = q.tally_votes_slots(int(cfg[g]) & 0xFFFF, int(cfg[g]) >> 16, pre[g])
        assert (gr_[g], rj_[g], res[g]) == (eg, er, eres), g


@pytest.mark.parametrize("prevote", [False, True])
@pytest.mark.parametrize("G,M,seed", [(500, 3000, 1), (4000, 20000, 2), (50, 5000, 3)])
def test_record_votes_vs_sequential(prevote, G, M, seed):
    _run(prevote, G, M, seed)


def test_election_table_through_record_votes(tables):
    """TestLeaderElectionInOneRoundRPC (raft_paper_test.go:192-232): the
    candidate's self vote then the table's responses, via RecordVote + Tally."""
    want = {"StateLeader": VoteResult.VoteWon, "StateFollower": VoteResult.VoteLost,
            "StateCandidate": VoteResult.VotePending}
    cases = tables["TestLeaderElectionInOneRoundRPC"]["cases"]
    cc = batch.compile_configs([range(1, tc["size"] + 1) for tc in cases])
    grp = batch.CsrGroups.from_compiled(cc, np.zeros(len(cc.slot_ids), np.uint64), device=DEV)
    group, slot, reject = [], [], []
    for g, tc in enumerate(cases):
        group.append(g), slot.append(0), reject.append(False)  # poll(r.id, ..., true), raft.go:803
        for vid, v in tc["votes"].items():
            group.append(g), slot.append(int(vid) - 1), reject.append(not v)
    M = len(group)
    term = np.ones(M, np.uint64)
    b = batch.AppRespBatch.from_numpy(group, slot, np.zeros(M, np.uint64), term, reject,
                                      device=DEV)
    grp.record_votes(b, batch.from_u64(np.ones(len(cases), np.uint64), DEV))
    _, _, res = grp.tally_votes()
    assert [VoteResult(int(x)) for x in res.cpu().numpy()] == [want[tc["state"]] for tc in cases]
