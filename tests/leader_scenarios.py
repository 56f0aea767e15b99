"""Replays the transcribed reference scenarios (tests/golden/leader_tables.json)
through an engine — the CPU oracle here, the HIP engine in test_gpu_leader.py —
and checks the expectations the reference tests assert."""
from __future__ import annotations

import json
import os

from oracle import leader_ref as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_tables():
    with open(os.path.join(ROOT, "tests", "golden", "leader_tables.json"), encoding="utf-8") as f:
        return json.load(f)


def build_group(sc) -> L.LeaderGroup:
    lg = sc["log"]
    log = L.LogView(first=lg["first"], last=lg["last"], committed=lg["committed"],
                    runs=[tuple(r) for r in lg["runs"]], snap_index=lg["snap_index"],
                    snap_term=lg["snap_term"], max_ents=lg["max_ents"])
    prs = []
    for p in sc["progress"]:
        infl = L.Inflights(sc["infl_size"])
        for v in p["infl"]:
            infl.add(v)
        prs.append(L.Progress(match=p["match"], next=p["next"], state=p["state"],
                              pending_snapshot=p["pending_snapshot"],
                              recent_active=p["recent_active"], probe_sent=p["probe_sent"],
                              inflights=infl))
    readq = [L.ReadIndexStatus(r["ctx"], r["index"], set(r["acks"]), r["from"]) for r in sc["readq"]]
    return L.LeaderGroup(sc["slots"], sc["mask_in"], sc["mask_out"], sc["term"], sc["leader"],
                         log, prs, transferee=sc["transferee"], read_only=sc["read_only"],
                         readq=readq)


def inbound(op) -> L.Inbound:
    """One inbound record of a scenario ('recv' op or a 'recv_batch' entry)."""
    return L.Inbound(kind=op["kind"], slot=op["slot"], term=op["term"], index=op["index"],
                     reject=op["reject"], hint=op["hint"], log_term=op["log_term"])


MSG_FIELDS = ("type", "to", "index", "log_term", "commit", "aux")


def check_expect(where, exp, msgs, group: L.LeaderGroup):
    """msgs: list of dicts with MSG_FIELDS; group: the state after the op."""
    if "n_msgs" in exp:
        assert len(msgs) == exp["n_msgs"], f"{where}: {len(msgs)} msgs, want {exp['n_msgs']}: {msgs}"
    for j, want in enumerate(exp.get("msgs", [])):
        assert j < len(msgs), f"{where}: missing msg {j}"
        for k, v in want.items():
            assert msgs[j][k] == v, f"{where}: msg {j} {k}={msgs[j][k]}, want {v}"
    for k, v in exp.get("all_msgs", {}).items():
        for j, m in enumerate(msgs):
            assert m[k] == v, f"{where}: msg {j} {k}={m[k]}, want {v}"
    for slot, want in exp.get("progress", {}).items():
        p = group.prs[int(slot)]
        for k, v in want.items():
            assert getattr(p, k) == v, f"{where}: progress[{slot}].{k}={getattr(p, k)}, want {v}"
    if "committed" in exp:
        assert group.log.committed == exp["committed"], f"{where}: committed {group.log.committed}"
    if "msgs_exact" in exp:
        got = [[m[k] for k in MSG_FIELDS] for m in msgs]
        assert got == exp["msgs_exact"], f"{where}: msgs {got}, want {exp['msgs_exact']}"
    if "status" in exp:
        got = [group.progress_string(s) for s in range(group.n_slots)]
        assert got == exp["status"], f"{where}: status {got}, want {exp['status']}"
    if "readq_len" in exp:
        assert len(group.readq) == exp["readq_len"], f"{where}: readq {group.readq}"


def msg_dict(m: L.Msg):
    return {"type": m.type, "to": m.to, "index": m.index, "log_term": m.log_term,
            "commit": m.commit, "aux": m.aux}


def run_scenario_oracle(sc):
    g = build_group(sc)
    for k, op in enumerate(sc["ops"]):
        g.msgs = []
        if op["op"] == "recv":
            g.step(inbound(op), k)
        elif op["op"] == "recv_batch":
            for j, m in enumerate(op["msgs"]):
                g.step(inbound(m), j)
        else:
            g.propose(op["n"])
        check_expect(f"{sc['name']} op{k}", op["expect"], [msg_dict(m) for m in g.msgs], g)
    return g
