"""Pin the CPU oracle to the reference's own known answers (no GPU needed).

* 127 datadriven cases (raft/quorum/testdata/*.txt, harness
  raft/quorum/datadriven_test.go:36-250): full expected output text,
  including Describe() and the harness's internal consistency checks.
* TestCommit (raft/raft_test.go:1127-1174), TestLeaderElectionInOneRoundRPC
  (raft/raft_paper_test.go:192-232), TestProgressUpdate
  (raft/tracker/progress_test.go:149-179).
"""
import random

import pytest

from oracle import quorum_ref as q

MAX = q.MAX_U64


def test_golden_count(golden):
    assert golden["count"] == 127
    by_file = {}
    for c in golden["cases"]:
        by_file[c["file"]] = by_file.get(c["file"], 0) + 1
    # 16 majority-commit, 22 majority-vote, 50 joint-commit, 39 joint-vote
    assert by_file == {"majority_commit.txt": 16, "majority_vote.txt": 22,
                       "joint_commit.txt": 50, "joint_vote.txt": 39}


def test_datadriven_full_output(golden):
    bad = [(c["file"], c["line"]) for c in golden["cases"]
           if q.datadriven_output(c) != c["expected_output"]]
    assert not bad, bad


def _log_term_of(log):
    terms = {i: t for i, t in log}
    last = max(terms) if terms else 0
    return lambda i: terms.get(i, 0) if 1 <= i <= last else 0


def test_commit_table(tables):
    for k, tc in enumerate(tables["TestCommit"]["cases"]):
        ids = set(range(1, len(tc["matches"]) + 1))
        acked = {i + 1: m for i, m in enumerate(tc["matches"])}
        ci = q.majority_committed_index(ids, acked)
        got = q.log_maybe_commit(0, ci, tc["term"], _log_term_of(tc["log"]))
        assert got == tc["want"], (k, tc)


def test_commit_table_window_form(tables):
    """The kernels' term gate (ci >= term_start) equals the
    log-based term(ci) == Term check on every TestCommit case."""
    for k, tc in enumerate(tables["TestCommit"]["cases"]):
        ids = set(range(1, len(tc["matches"]) + 1))
        acked = {i + 1: m for i, m in enumerate(tc["matches"])}
        ci = q.majority_committed_index(ids, acked)
        same = [i for i, t in tc["log"] if t == tc["term"]]
        term_start = min(same) if same else MAX
        last = max(i for i, _ in tc["log"])
        assert ci <= last
        gated = ci if (ci > 0 and ci >= term_start) else 0
        assert gated == tc["want"], (k, tc)


def test_election_table(tables):
    want = {"StateLeader": q.VOTE_WON, "StateFollower": q.VOTE_LOST,
            "StateCandidate": q.VOTE_PENDING}
    for k, tc in enumerate(tables["TestLeaderElectionInOneRoundRPC"]["cases"]):
        votes = {1: True}  # the candidate votes for itself (raft.go:803)
        votes.update({int(i): v for i, v in tc["votes"].items()})
        r = q.joint_vote_result(set(range(1, tc["size"] + 1)), set(), votes)
        assert r == want[tc["state"]], (k, tc)


def test_progress_update_table(tables):
    t = tables["TestProgressUpdate"]
    for k, tc in enumerate(t["cases"]):
        m, n, ok = q.progress_maybe_update(t["prev_match"], t["prev_next"], tc["update"])
        assert (m, n, ok) == (tc["wm"], tc["wn"], tc["wok"]), (k, tc)


def _quick_map(rng, size=10):
    """smallRandIdxMap (quick_test.go:47-64)."""
    n = rng.randrange(size)
    ids = rng.sample(range(2 * n), n) if n else []
    return {i: rng.randrange(n) for i in ids}


def test_quick_alternative():
    """TestQuick (quick_test.go:28-45): CommittedIndex == the counting form."""
    rng = random.Random(1)
    for _ in range(5000):
        c = set(_quick_map(rng))
        l = _quick_map(rng)
        assert q.majority_committed_index(c, l) == q.alternative_majority_committed_index(c, l)


@pytest.mark.parametrize("seed", range(3))
def test_joint_invariants(seed):
    """datadriven_test.go:175-240 invariants on random inputs: zero-joint,
    self-joint, symmetry, overlay-lowering."""
    rng = random.Random(seed)
    for _ in range(2000):
        c0 = set(_quick_map(rng))
        c1 = set(_quick_map(rng))
        l = {i: rng.randrange(1, 50) for i in c0 | c1 if rng.random() < 0.8}
        ci = q.majority_committed_index(c0, l)
        assert q.joint_committed_index(c0, set(), l) == ci
        assert q.joint_committed_index(c0, c0, l) == ci
        assert q.joint_committed_index(c0, c1, l) == q.joint_committed_index(c1, c0, l)
        votes = {i: rng.random() < 0.5 for i in c0 | c1 if rng.random() < 0.7}
        assert q.joint_vote_result(c0, c1, votes) == q.joint_vote_result(c1, c0, votes)
        for vid in c0:
            v = l.get(vid, 0)
            if ci > v > 0:
                lo = dict(l)
                lo[vid] = v - 1
                assert q.majority_committed_index(c0, lo) == ci
