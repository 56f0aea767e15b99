#!/usr/bin/env python3
"""Write tests/golden/leader_tables.json: the reference's own tests for the
leader inbox step transcribed as data.

Everything below is inputs and expected outputs read off the reference's test
files (paths relative to the reference's raft/); the setup each scenario
starts from is the state the cited test builds before its first Step, restated
as Progress / log fields (becomeLeader -> reset: peers Probe with Match 0 and
Next = lastIndex+1, the leader Replicate with Match = lastIndex after it
appends its empty entry at the new term; raft.go:590-620, 725-760).  Messages
the tests Step without a Term are local (Term 0, raft.go:849-850).

Slot s is voter ID s+1 (IDs 1..n).  Nothing here is executed against the
reference at test time; the JSON is committed.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
UNLIMITED = 1 << 62  # MaxSizePerMsg: noLimit (raft_test.go:4808)

P, R, S = 0, 1, 2                    # StateProbe / StateReplicate / StateSnapshot
APP, HB, SNAPST, UNREACH = 0, 1, 2, 3  # inbound kinds
MSG_APP, MSG_SNAP, MSG_TIMEOUT_NOW, MSG_READ_INDEX_RESP = 3, 7, 14, 16


def runs_of(terms):
    """Term runs of a log whose entry i (1-based) has terms[i-1]; index 0 is
    the dummy entry with term 0."""
    runs = [[0, 0]]
    for i, t in enumerate(terms, start=1):
        if t != runs[-1][1]:
            runs.append([i, t])
    return runs


def pr(match, nxt, state=P, probe_sent=False, recent_active=False, pending_snapshot=0, infl=()):
    return {"match": match, "next": nxt, "state": state, "probe_sent": probe_sent,
            "recent_active": recent_active, "pending_snapshot": pending_snapshot,
            "infl": list(infl)}


def recv(kind, slot, term=0, index=0, reject=False, hint=0, log_term=0, expect=None):
    return {"op": "recv", "kind": kind, "slot": slot, "term": term, "index": index,
            "reject": reject, "hint": hint, "log_term": log_term, "expect": expect or {}}


def leader_after_election(n, log_terms, term, committed=0, infl_size=256, max_ents=UNLIMITED):
    """State right after becomeCandidate + becomeLeader on a fresh node whose
    storage holds ``log_terms``: the empty entry of ``term`` is appended."""
    last0 = len(log_terms)
    terms = list(log_terms) + [term]
    prs = [pr(0, last0 + 1) for _ in range(n)]
    prs[0] = pr(last0 + 1, last0 + 2, state=R)
    return {"slots": n, "mask_in": (1 << n) - 1, "mask_out": 0, "term": term, "leader": 0,
            "transferee": 255, "read_only": 0, "infl_size": infl_size,
            "log": {"first": 1, "last": len(terms), "committed": committed,
                    "runs": runs_of(terms), "snap_index": 0, "snap_term": 0,
                    "max_ents": max_ents},
            "progress": prs, "readq": [], "ops": []}


def scenarios():
    out = []

    # TestLeaderAppResp (raft_test.go:2426-2482).  Storage ents {1,t0} {2,t1}
    # and unstable offset 3; the leader's empty entry is index 3 at term 1.
    for i, (index, reject, wmatch, wnext, wmsg, windex, wcommit) in enumerate([
            (3, True, 0, 3, 0, 0, 0),
            (2, True, 0, 2, 1, 1, 0),
            (2, False, 2, 4, 2, 2, 2),
            (0, False, 0, 3, 0, 0, 0)]):
        sc = leader_after_election(3, [0, 1], 1)
        sc["name"] = f"TestLeaderAppResp#{i}"
        sc["cite"] = "raft/raft_test.go:2426-2482"
        sc["ops"].append(recv(APP, 1, term=1, index=index, reject=reject, hint=index, expect={
            "progress": {"1": {"match": wmatch, "next": wnext}},
            "n_msgs": wmsg, "all_msgs": {"index": windex, "commit": wcommit}}))
        out.append(sc)

    # TestFastLogRejection (raft_test.go:4319-4600), leader side: after the
    # heartbeat response the leader probes at its old last index; the
    # follower's rejection (hint index/term, asserted by the test) must make
    # the next MsgApp carry (nextAppendIndex, nextAppendTerm).
    fast = [
        ([1, 2, 2, 4, 4, 4, 4], 3, 7, 2, 3),
        ([1, 2, 2, 3, 4, 4, 4, 5], 3, 8, 3, 4),
        ([1, 1, 1, 1], 1, 1, 1, 1),
        ([1, 1, 1, 1, 1, 1], 1, 1, 1, 1),
        ([1, 1, 1, 1], 1, 1, 1, 1),
        ([1, 1, 1, 4, 5], 4, 4, 4, 4),
        ([2, 5, 5, 5, 5, 5, 5, 5, 5], 4, 6, 2, 1),
        ([2, 2, 2, 2, 2], 2, 1, 2, 1),
    ]
    for i, (leader_log, hint_term, hint_index, next_term, next_index) in enumerate(fast):
        sc = leader_after_election(3, leader_log, 1)
        sc["name"] = f"TestFastLogRejection#{i}"
        sc["cite"] = "raft/raft_test.go:4319-4600"
        L = len(leader_log)
        sc["ops"].append(recv(HB, 1, expect={"n_msgs": 1, "msgs": [{"type": MSG_APP}]}))
        sc["ops"].append(recv(APP, 1, term=1, index=L, reject=True, hint=hint_index,
                              log_term=hint_term,
                              expect={"msgs": [{"type": MSG_APP, "index": next_index,
                                                "log_term": next_term}]}))
        out.append(sc)

    # TestProgressFlowControl (raft_test.go:111-180): MaxInflightMsgs 3,
    # MaxSizePerMsg 2048 with 1000-byte entries (two per MsgApp).  Entry 1 is
    # the election's empty entry, 2..11 the ten proposals; node 2 was probed
    # with [1,2] and is paused (ProbeSent).
    sc = leader_after_election(2, [], 1, infl_size=3, max_ents=2)
    sc["name"] = "TestProgressFlowControl"
    sc["cite"] = "raft/raft_test.go:111-180"
    sc["log"]["last"] = 11
    sc["progress"][0] = pr(11, 12, state=R)
    sc["progress"][1] = pr(0, 1, state=P, probe_sent=True)
    sc["ops"].append(recv(APP, 1, index=2, expect={
        "n_msgs": 3, "all_msgs": {"type": MSG_APP, "aux": 2}}))
    sc["ops"].append(recv(APP, 1, index=8, expect={
        "n_msgs": 2, "msgs": [{"type": MSG_APP, "aux": 2}, {"type": MSG_APP, "aux": 1}]}))
    out.append(sc)

    # TestSendAppendForProgressProbe (raft_test.go:2613-2678), last step: 31
    # proposals after the election entry, node 2 probed at index 0 and paused;
    # a heartbeat response lets exactly one more probe out.
    sc = leader_after_election(2, [], 1)
    sc["name"] = "TestSendAppendForProgressProbe"
    sc["cite"] = "raft/raft_test.go:2613-2678"
    sc["log"]["last"] = 32
    sc["progress"][0] = pr(32, 33, state=R)
    sc["progress"][1] = pr(0, 1, state=P, probe_sent=True)
    sc["ops"].append(recv(HB, 1, expect={
        "n_msgs": 1, "msgs": [{"index": 0}], "progress": {"1": {"probe_sent": True}}}))
    out.append(sc)

    # TestHandleHeartbeatResp (raft_test.go:1312-1357): storage {1,t1} {2,t2}
    # {3,t3}; the election entry is 4 at term 1 and is committed.
    sc = leader_after_election(2, [1, 2, 3], 1, committed=4)
    sc["name"] = "TestHandleHeartbeatResp"
    sc["cite"] = "raft/raft_test.go:1312-1357"
    sc["ops"].append(recv(HB, 1, expect={"n_msgs": 1, "msgs": [{"type": MSG_APP}]}))
    sc["ops"].append(recv(HB, 1, expect={"n_msgs": 1, "msgs": [{"type": MSG_APP}]}))
    sc["ops"].append(recv(APP, 1, index=3 + 1, expect={}))  # msgs[0].Index + len(Entries)
    sc["ops"].append(recv(HB, 1, expect={"n_msgs": 0}))
    out.append(sc)

    # TestMsgAppRespWaitReset (raft_test.go:1407-1465): three voters, the
    # election entry 1 at term 1 already broadcast (both followers probed and
    # paused).
    sc = leader_after_election(3, [], 1)
    sc["name"] = "TestMsgAppRespWaitReset"
    sc["cite"] = "raft/raft_test.go:1407-1465"
    sc["progress"][1] = pr(0, 1, state=P, probe_sent=True)
    sc["progress"][2] = pr(0, 1, state=P, probe_sent=True)
    sc["ops"].append(recv(APP, 1, index=1, expect={"committed": 1}))
    sc["ops"].append({"op": "propose", "n": 1, "expect": {
        "n_msgs": 1, "msgs": [{"type": MSG_APP, "to": 1, "aux": 1, "index": 1}]}})
    sc["ops"].append(recv(APP, 2, index=1, expect={
        "n_msgs": 1, "msgs": [{"type": MSG_APP, "to": 2, "aux": 1, "index": 1}]}))
    out.append(sc)

    # TestRecvMsgUnreachable (raft_test.go:2714-2737): storage {1..3, t1};
    # node 2 Match 3, Replicate, OptimisticUpdate(5).
    sc = leader_after_election(2, [1, 1, 1], 1)
    sc["name"] = "TestRecvMsgUnreachable"
    sc["cite"] = "raft/raft_test.go:2714-2737"
    sc["progress"][1] = pr(3, 6, state=R)
    sc["ops"].append(recv(UNREACH, 1, expect={"progress": {"1": {"state": P, "next": 4}}}))
    out.append(sc)

    # TestRaftFreesReadOnlyMem (raft_test.go:1359-1405): the election entry is
    # committed; node 2's MsgReadIndex("ctx") was queued at index 1 with the
    # leader's own ack (sendMsgReadIndexResponse, raft.go:1827-1837).
    sc = leader_after_election(2, [], 1, committed=1)
    sc["name"] = "TestRaftFreesReadOnlyMem"
    sc["cite"] = "raft/raft_test.go:1359-1405"
    ctx = int.from_bytes(b"ctx", "little")
    sc["readq"] = [{"ctx": ctx, "index": 1, "acks": [0], "from": 1}]
    sc["ops"].append(recv(HB, 1, index=ctx, expect={"readq_len": 0}))
    out.append(sc)
    return out


def batch(msgs, expect_msgs=None, **exp):
    """One inbound batch (an interaction test's '> 1 receiving messages' block)
    and the leader's outbound messages in its next Ready (exactly, in order)."""
    e = dict(exp)
    if expect_msgs is not None:
        e["msgs_exact"] = expect_msgs
    return {"op": "recv_batch", "msgs": msgs, "expect": e}


def app(slot, index, term, reject=False, hint=0, log_term=0):
    return {"kind": APP, "slot": slot, "term": term, "index": index, "reject": reject,
            "hint": hint, "log_term": log_term}


def hb(slot, term, ctx=0):
    return {"kind": HB, "slot": slot, "term": term, "index": ctx, "reject": False, "hint": 0,
            "log_term": 0}


def mapp(to, index, log_term, commit, n):
    return [MSG_APP, to, index, log_term, commit, n]


def interaction_scenarios():
    """Leader side of the reference's interaction tests (raft/testdata/*.txt,
    run by raft/interaction_test.go:24-34 through rafttest's InteractionEnv):
    every '> 1 receiving messages' block is one batch, the following
    '> 1 handling Ready' block's Messages (or none) its expected output; the
    'status 1' blocks are Progress.String() of every peer.  Node i is slot
    i-1.  The env's raft.Config (rafttest/interaction_env.go:90-99) has
    MaxSizePerMsg = MaxUint64 and MaxInflightMsgs = MaxInt32 (never full)."""
    out = []
    # probe_and_replicate.txt:470-767: n1 became leader at term 8 over the
    # Figure-7 log (shifted by 10: snapshot index 10 term 1, entries 11..20 of
    # terms 1 1 1 4 4 5 5 6 6 6, its empty entry 21 at term 8), commit 18, and
    # probed every peer at Log:6/20 (all Probe, Next 21, ProbeSent).
    sc = {"name": "interaction/probe_and_replicate", "cite": "raft/testdata/probe_and_replicate.txt:470-767",
          "slots": 7, "mask_in": 0x7F, "mask_out": 0, "term": 8, "leader": 0, "transferee": 255,
          "read_only": 0, "infl_size": 16,
          "log": {"first": 11, "last": 21, "committed": 18,
                  "runs": [[10, 1], [14, 4], [16, 5], [18, 6], [21, 8]],
                  "snap_index": 10, "snap_term": 1, "max_ents": UNLIMITED},
          "progress": [pr(21, 22, state=R)] + [pr(0, 21, probe_sent=True) for _ in range(6)],
          "readq": [], "ops": []}
    ops = sc["ops"]
    for node, (hint_term, hint), (lt, idx, n) in (
            (2, (6, 19), (6, 19, 2)), (3, (4, 14), (4, 14, 7))):
        s_ = node - 1
        ops.append(batch([app(s_, 20, 8, True, hint, hint_term)], [mapp(s_, idx, lt, 18, n)]))
        ops.append(batch([app(s_, 21, 8)], [mapp(s_, 21, 8, 18, 0)]))
        ops.append(batch([app(s_, 21, 8)], []))
    ops.append(batch([app(3, 21, 8)], [mapp(1, 21, 8, 21, 0), mapp(2, 21, 8, 21, 0),
                                       mapp(3, 21, 8, 21, 0)], committed=21))
    ops.append(batch([app(3, 21, 8)], []))
    for node, (hint_term, hint), (lt, idx, n) in (
            (5, (6, 18), (6, 18, 3)), (6, (4, 17), (4, 15, 6)), (7, (3, 20), (1, 13, 8))):
        s_ = node - 1
        ops.append(batch([app(s_, 20, 8, True, hint, hint_term)], [mapp(s_, idx, lt, 21, n)]))
        ops.append(batch([app(s_, 21, 8)], [mapp(s_, 21, 8, 21, 0)]))
        ops.append(batch([app(s_, 21, 8)], []))
    out.append(sc)

    # snapshot_succeed_via_app_resp.txt: n1 leads at term 1 over voters 1-3
    # with everything up to 11 replicated to n2 and compacted away
    # (firstIndex 12, snapshot index 11 term 1); n3 never answered.
    sc = {"name": "interaction/snapshot_succeed_via_app_resp",
          "cite": "raft/testdata/snapshot_succeed_via_app_resp.txt:36-125",
          "slots": 3, "mask_in": 0x7, "mask_out": 0, "term": 1, "leader": 0, "transferee": 255,
          "read_only": 0, "infl_size": 16,
          "log": {"first": 12, "last": 11, "committed": 11, "runs": [[11, 1]],
                  "snap_index": 11, "snap_term": 1, "max_ents": UNLIMITED},
          "progress": [pr(11, 12, state=R), pr(11, 12, state=R, recent_active=True),
                       pr(0, 11, probe_sent=True)],
          "readq": [], "ops": []}
    sc["ops"].append(batch([], [], status=["StateReplicate match=11 next=12 inactive",
                                           "StateReplicate match=11 next=12",
                                           "StateProbe match=0 next=11 paused inactive"]))
    sc["ops"].append(batch([hb(2, 1)], [[MSG_SNAP, 2, 11, 1, 0, 0]],
                           status=["StateReplicate match=11 next=12 inactive",
                                   "StateReplicate match=11 next=12",
                                   "StateSnapshot match=0 next=11 paused pendingSnap=11"]))
    sc["ops"].append(batch([app(2, 11, 1)], [mapp(2, 11, 1, 11, 0)],
                           status=["StateReplicate match=11 next=12 inactive",
                                   "StateReplicate match=11 next=12",
                                   "StateReplicate match=11 next=12"]))
    sc["ops"].append(batch([hb(1, 1), app(2, 11, 1)], []))
    out.append(sc)
    return out


def progress_tables():
    return {
        # tracker/progress_test.go:40-66
        "TestProgressIsPaused": [[P, False, False], [P, True, True], [R, False, False],
                                 [R, True, False], [S, False, True], [S, True, True]],
        # tracker/progress_test.go:84-117: match 1; (state, next, pendingSnapshot, wnext)
        "TestProgressBecomeProbe": [[R, 5, 0, 2], [S, 5, 10, 11], [S, 5, 0, 2]],
        # tracker/progress_test.go:119-132 / 134-147
        "TestProgressBecomeReplicate": {"match": 1, "next": 5, "wnext": 2},
        "TestProgressBecomeSnapshot": {"match": 1, "next": 5, "snap": 10},
        # tracker/progress_test.go:181-250: (state, m, n, rejected, last, w, wn)
        "TestProgressMaybeDecr": [
            [R, 5, 10, 5, 5, False, 10], [R, 5, 10, 4, 4, False, 10],
            [R, 5, 10, 9, 9, True, 6], [P, 0, 0, 0, 0, False, 0],
            [P, 0, 10, 5, 5, False, 10], [P, 0, 10, 9, 9, True, 9],
            [P, 0, 2, 1, 1, True, 1], [P, 0, 1, 0, 0, True, 1],
            [P, 0, 10, 9, 2, True, 3], [P, 0, 10, 9, 0, True, 1]],
        # tracker/progress_test.go:68-82
        "TestProgressResume": {"next": 2, "decr": [1, 1], "update": 2},
    }


def inflight_tables():
    # tracker/inflights_test.go: op sequences with the expected
    # (start, count, buffer) after each "expect".
    return [
        {"name": "TestInflightsAdd/no-rotate", "size": 10, "start": 0, "ops": [
            ["add", [0, 1, 2, 3, 4]], ["expect", 0, 5, [0, 1, 2, 3, 4, 0, 0, 0, 0, 0]],
            ["add", [5, 6, 7, 8, 9]], ["expect", 0, 10, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]]]},
        {"name": "TestInflightsAdd/rotate", "size": 10, "start": 5, "ops": [
            ["add", [0, 1, 2, 3, 4]], ["expect", 5, 5, [0, 0, 0, 0, 0, 0, 1, 2, 3, 4]],
            ["add", [5, 6, 7, 8, 9]], ["expect", 5, 10, [5, 6, 7, 8, 9, 0, 1, 2, 3, 4]]]},
        {"name": "TestInflightFreeTo", "size": 10, "start": 0, "ops": [
            ["add", list(range(10))], ["free_le", 4],
            ["expect", 5, 5, list(range(10))], ["free_le", 8],
            ["expect", 9, 1, list(range(10))], ["add", [10, 11, 12, 13, 14]], ["free_le", 12],
            ["expect", 3, 2, [10, 11, 12, 13, 14, 5, 6, 7, 8, 9]], ["free_le", 14],
            ["expect", 0, 0, [10, 11, 12, 13, 14, 5, 6, 7, 8, 9]]]},
        {"name": "TestInflightFreeFirstOne", "size": 10, "start": 0, "ops": [
            ["add", list(range(10))], ["free_first_one"],
            ["expect", 1, 9, list(range(10))]]},
    ]


def main():
    doc = {"scenarios": scenarios() + interaction_scenarios(), "progress": progress_tables(),
           "inflights": inflight_tables()}
    with open(os.path.join(HERE, "leader_tables.json"), "w", encoding="utf-8") as f:
        json.dump(doc, f, indent=1)
    print("wrote", len(doc["scenarios"]), "scenarios")


if __name__ == "__main__":
    main()
