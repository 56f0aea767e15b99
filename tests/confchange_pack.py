"""Packing between the confchange oracle's Trackers and the engine's CSR
config + Progress arrays; random tracker/ops generators.  Test infrastructure."""
import random

import numpy as np

from oracle import confchange_ref as CC


def pack(trackers):
    off = [0]
    ids, match, nxt, psnap, pst, ipos = [], [], [], [], [], []
    cfg, ext = [], []
    for t in trackers:
        slots = sorted(t.prs)
        mi = mo = ln = 0
        for j, i in enumerate(slots):
            p = t.prs[i]
            mi |= (i in t.voters_in) << j
            mo |= (i in (t.voters_out or ())) << j
            ln |= (i in (t.learners_next or ())) << j
            ids.append(i)
            match.append(p.match)
            nxt.append(p.next)
            psnap.append(p.pending_snapshot)
            pst.append(p.state | (4 if p.probe_sent else 0) | (8 if p.recent_active else 0))
            ipos.append(p.inflight_count << 16)
        cfg.append(mi | (mo << 16))
        ext.append(ln | ((1 << 16) if t.auto_leave else 0))
        off.append(off[-1] + len(slots))
    prog = {"match": np.array(match, np.uint64), "next": np.array(nxt, np.uint64),
            "pending_snapshot": np.array(psnap, np.uint64), "pstate": np.array(pst, np.uint8),
            "infl_pos": np.array(ipos, np.uint32)}
    return (np.array(off, np.uint32), np.array(ids, np.uint64), np.array(cfg, np.uint32),
            np.array(ext, np.uint32), prog)


def unpack(a, max_inflight):
    out = []
    off = a["off"]
    for g in range(len(a["cfg"])):
        c, e = int(a["cfg"][g]), int(a["ext"][g])
        vin, vout, ln, lr = set(), set(), set(), set()
        prs = {}
        for j, s in enumerate(range(int(off[g]), int(off[g + 1]))):
            i = int(a["ids"][s])
            bi, bo, bl = (c >> j) & 1, (c >> (16 + j)) & 1, (e >> j) & 1
            if bi:
                vin.add(i)
            if bo:
                vout.add(i)
            if bl:
                ln.add(i)
            learner = not (bi or bo or bl)
            if learner:
                lr.add(i)
            st = int(a["pstate"][s])
            prs[i] = CC.Pr(match=int(a["match"][s]), next=int(a["next"][s]), state=st & 3,
                           probe_sent=bool(st & 4), pending_snapshot=int(a["pending_snapshot"][s]),
                           recent_active=bool(st & 8), is_learner=learner,
                           inflight_count=int(a["infl_pos"][s]) >> 16, inflight_size=max_inflight)
        out.append(CC.Tracker(vin, vout or None, lr or None, ln or None, bool((e >> 16) & 1), prs,
                              max_inflight))
    return out


def random_ccs(r: random.Random, n_ids=8):
    k = r.choice([0, 1, 1, 1, 2, 3, 5])
    out = []
    for _ in range(k):
        typ = r.choice([CC.ADD_NODE, CC.ADD_NODE, CC.ADD_LEARNER, CC.REMOVE_NODE, CC.UPDATE_NODE])
        if r.random() < 0.02:
            typ = 7  # unknown type
        out.append((typ, r.choice(range(0 if r.random() < 0.05 else 1, n_ids + 1))))
    return out


def random_op(r: random.Random, t):
    joint = bool(t.voters_out)
    x = r.random()
    if joint:
        return 4 if x < 0.6 else (1 if x < 0.8 else 2)
    return 1 if x < 0.6 else (2 if x < 0.8 else (3 if x < 0.9 else 4))


def oracle_apply(t, op, ccs, last_index):
    ch = CC.Changer(t, last_index)
    if op == 0:
        return t, None
    try:
        if op == 1:
            return ch.simple(ccs), None
        if op in (2, 3):
            return ch.enter_joint(op == 3, ccs), None
        return ch.leave_joint(), None
    except CC.ConfChangeError as e:
        return t, str(e)
