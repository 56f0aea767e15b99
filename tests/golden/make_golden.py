#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference's own test data.

Run here (where /root/reference exists); the JSON it writes is committed and is
what every test reads, so nothing at test time touches /root/reference.

Outputs
-------
tests/golden/quorum_datadriven.json
    The 127 known-answer cases of ``TestDataDriven``
    (raft/quorum/datadriven_test.go:36-250) parsed out of
    raft/quorum/testdata/{majority,joint}_{commit,vote}.txt.  Each case keeps the
    command, its arguments and the full expected output text (Describe() lines
    plus the result on the last line).  The datadriven text format
    (github.com/cockroachdb/datadriven @ v0.0.0-20200714090401-bf6692d28da5,
    not vendored in the reference) is: optional ``#`` comments, one command
    line, ``----``, the expected output up to the next blank line.

tests/golden/raft_tables.json
    Table tests transcribed as data (inputs and expected outputs only):
      * TestCommit                        raft/raft_test.go:1127-1174
      * TestLeaderElectionInOneRoundRPC   raft/raft_paper_test.go:192-232
      * TestProgressUpdate                raft/tracker/progress_test.go:149-179
"""
import json
import os
import re
import sys

REF = "/root/reference/raft"
HERE = os.path.dirname(os.path.abspath(__file__))

ARG_RE = re.compile(r"(\w+)(?:=(\([^)]*\)|\S+))?")


def parse_args(s):
    out = []
    for m in ARG_RE.finditer(s):
        key, val = m.group(1), m.group(2)
        if val is None:
            vals = []
        elif val.startswith("("):
            vals = [v.strip() for v in val[1:-1].split(",") if v.strip() != ""]
        else:
            vals = [val]
        out.append((key, vals))
    return out


def parse_datadriven(path):
    cases = []
    lines = open(path, encoding="utf-8").read().split("\n")
    i = 0
    while i < len(lines):
        ln = lines[i]
        if ln.strip() == "" or ln.startswith("#"):
            i += 1
            continue
        cmdline = ln
        pos = i + 1
        assert lines[i + 1] == "----", (path, i, ln)
        i += 2
        out = []
        while i < len(lines) and lines[i] != "":
            out.append(lines[i])
            i += 1
        parts = cmdline.split(None, 1)
        cmd = parts[0]
        args = parse_args(parts[1]) if len(parts) > 1 else []
        case = {"file": os.path.basename(path), "line": pos, "cmd": cmd,
                "cfg": [], "cfgj": None, "idx": [], "votes": []}
        for key, vals in args:
            if key == "cfg":
                case["cfg"] += [int(v) for v in vals]
            elif key == "cfgj":
                if vals == ["zero"]:
                    case["cfgj"] = []
                else:
                    case["cfgj"] = (case["cfgj"] or []) + [int(v) for v in vals]
            elif key == "idx":
                case["idx"] += [None if v == "_" else int(v) for v in vals]
            elif key == "votes":
                case["votes"] += [{"y": 2, "n": 1, "_": 0}[v] for v in vals]
            else:
                raise ValueError(f"unknown arg {key} in {path}:{pos}")
        case["expected_output"] = "\n".join(out) + "\n"
        case["expected_result"] = out[-1] if out else ""
        cases.append(case)
    return cases


def tables():
    # TestCommit (raft/raft_test.go:1127-1174): matches, log (index, term),
    # smTerm, expected committed.
    commit = [
        ([1], [(1, 1)], 1, 1),
        ([1], [(1, 1)], 2, 0),
        ([2], [(1, 1), (2, 2)], 2, 2),
        ([1], [(1, 2)], 2, 1),
        ([2, 1, 1], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 2], [(1, 1), (2, 2)], 2, 2),
        ([2, 1, 2], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 1, 1], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1, 1], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 1, 2], [(1, 1), (2, 2)], 1, 1),
        ([2, 1, 1, 2], [(1, 1), (2, 1)], 2, 0),
        ([2, 1, 2, 2], [(1, 1), (2, 2)], 2, 2),
        ([2, 1, 2, 2], [(1, 1), (2, 1)], 2, 0),
    ]
    # TestLeaderElectionInOneRoundRPC (raft/raft_paper_test.go:192-232):
    # cluster size, votes received by candidate 1 (it also votes for itself,
    # raft.go:803), expected state.
    election = [
        (1, {}, "StateLeader"),
        (3, {2: True, 3: True}, "StateLeader"),
        (3, {2: True}, "StateLeader"),
        (5, {2: True, 3: True, 4: True, 5: True}, "StateLeader"),
        (5, {2: True, 3: True, 4: True}, "StateLeader"),
        (5, {2: True, 3: True}, "StateLeader"),
        (3, {2: False, 3: False}, "StateFollower"),
        (5, {2: False, 3: False, 4: False, 5: False}, "StateFollower"),
        (5, {2: True, 3: False, 4: False, 5: False}, "StateFollower"),
        (3, {}, "StateCandidate"),
        (5, {2: True}, "StateCandidate"),
        (5, {2: False, 3: False}, "StateCandidate"),
        (5, {}, "StateCandidate"),
    ]
    # TestProgressUpdate (raft/tracker/progress_test.go:149-179).
    prev_m, prev_n = 3, 5
    update = [
        (prev_m - 1, prev_m, prev_n, False),
        (prev_m, prev_m, prev_n, False),
        (prev_m + 1, prev_m + 1, prev_n, True),
        (prev_m + 2, prev_m + 2, prev_n + 1, True),
    ]
    return {
        "TestCommit": {
            "source": "raft/raft_test.go:1127-1174",
            "cases": [{"matches": m, "log": [list(e) for e in lg], "term": t, "want": w}
                      for m, lg, t, w in commit],
        },
        "TestLeaderElectionInOneRoundRPC": {
            "source": "raft/raft_paper_test.go:192-232",
            "cases": [{"size": s, "votes": {str(k): v for k, v in vt.items()}, "state": st}
                      for s, vt, st in election],
        },
        "TestProgressUpdate": {
            "source": "raft/tracker/progress_test.go:149-179",
            "prev_match": prev_m, "prev_next": prev_n,
            "cases": [{"update": u, "wm": wm, "wn": wn, "wok": ok} for u, wm, wn, ok in update],
        },
    }


def main():
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: the committed fixtures are authoritative")
    cases = []
    for name in ("majority_commit.txt", "majority_vote.txt", "joint_commit.txt", "joint_vote.txt"):
        cases += parse_datadriven(os.path.join(REF, "quorum", "testdata", name))
    doc = {
        "source": "raft/quorum/testdata/*.txt via raft/quorum/datadriven_test.go:36-250",
        "count": len(cases),
        "cases": cases,
    }
    with open(os.path.join(HERE, "quorum_datadriven.json"), "w", encoding="utf-8") as f:
        json.dump(doc, f, indent=1, ensure_ascii=False)
    with open(os.path.join(HERE, "raft_tables.json"), "w", encoding="utf-8") as f:
        json.dump(tables(), f, indent=1)
    print(f"wrote {len(cases)} datadriven cases")


if __name__ == "__main__":
    main()
