"""GPU parity of batched conf changes (qb_dev_conf_change) against the
confchange restatement: the reference's datadriven testdata replayed with
one group per file (outputs compared as the reference's text), random
operation sequences over many groups, and Restore(ConfState)."""
import json
import os
import random

import numpy as np
import pytest

from oracle import confchange_ref as CC
from tests import confchange_pack as CP

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DD = json.load(open(os.path.join(ROOT, "tests", "golden", "confchange_datadriven.json")))
OPS = {"simple": 1, "enter-joint": 2, "leave-joint": 4}


def _table(trackers, K=10):
    from etcd_amd.quorum.confchange import ConfigTable
    off, ids, cfg, ext, prog = CP.pack(trackers)
    return ConfigTable.from_numpy(off, ids, cfg, ext, prog, K)


def _render(t):
    return t.config_string() + "\n" + t.progress_string()


def test_datadriven_on_device():
    from etcd_amd.quorum.confchange import error_text
    names = sorted(DD)
    table = _table([CC.Tracker.empty(10) for _ in names])
    steps = max(len(DD[n]) for n in names)
    for k in range(steps):
        op, ccs, host_err = [], [], {}
        for g, n in enumerate(names):
            c = DD[n][k] if k < len(DD[n]) else None
            if c is None:
                op.append(0)
                ccs.append([])
                continue
            cc = CC.parse_ccs(c["input"])
            o = OPS[c["cmd"]]
            if o == 2 and c.get("autoleave"):
                o = 3
            if o == 4 and cc:
                host_err[g] = "this command takes no input"
                op.append(0)
                ccs.append([])
                continue
            op.append(o)
            ccs.append(cc)
        table, err, err_id = table.change(op, ccs, [k] * len(names))
        state = CP.unpack(table.numpy(), 10)
        for g, n in enumerate(names):
            if k >= len(DD[n]):
                continue
            c = DD[n][k]
            if g in host_err:
                got = host_err[g] + "\n"
            elif err[g]:
                got = error_text(int(err[g]), int(err_id[g])) + "\n"
            else:
                got = _render(state[g])
            assert got == c["expected"], f"{n}:{c['line']}\n{got}\nwant\n{c['expected']}"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_sequences(seed):
    from etcd_amd.quorum.confchange import error_text
    r = random.Random(seed)
    G = 600
    orc = [CC.Tracker.empty(7) for _ in range(G)]
    # random carried Progress content, so the copy of kept slots is checked
    table = _table(orc, K=7)
    for step in range(12):
        op = [CP.random_op(r, t) for t in orc]
        ccs = [CP.random_ccs(r) for _ in orc]
        last = [r.randint(0, 1000) for _ in orc]
        table, err, err_id = table.change(op, ccs, last)
        dev = CP.unpack(table.numpy(), 7)
        for g in range(G):
            nt, e = CP.oracle_apply(orc[g], op[g], ccs[g], last[g])
            if e is None and sum(1 for _ in nt.prs) > 16:
                e = "more than 16 members, or 24 alive within one change (engine limit)"
                nt = orc[g]
            got_e = error_text(int(err[g]), int(err_id[g])) if err[g] else None
            assert got_e == e, (seed, step, g, op[g], ccs[g], got_e, e)
            assert _render(dev[g]) == _render(nt), (seed, step, g)
            orc[g] = nt
        # perturb carried Progress on the device side and the oracle alike
        a = table.numpy()
        for g in range(G):
            for j, s in enumerate(range(int(a["off"][g]), int(a["off"][g + 1]))):
                i = int(a["ids"][s])
                v = r.randint(0, 99)
                a["match"][s] = v
                orc[g].prs[i].match = v
        from etcd_amd.quorum.confchange import ConfigTable
        table = ConfigTable.from_numpy(a["off"], a["ids"], a["cfg"], a["ext"],
                                       {k: a[k] for k in ("match", "next", "pending_snapshot",
                                                          "pstate", "infl_pos", "infl_buf")}, 7)


def test_churn_within_one_change_list():
    """a Simple change that adds and removes more than 8 learners in
    one list (the final config keeps its 5 voters) is legal in the reference;
    the device reuses the freed table entries instead of failing with the
    engine's slot limit.  Voters 1..5 are added one Simple change at a time
    first (each changes one voter)."""
    from etcd_amd.quorum.confchange import error_text
    G = 64
    orc = [CC.Tracker.empty(4) for _ in range(G)]
    table = _table(orc, K=4)
    plans = [[(CC.ADD_NODE, v)] for v in range(1, 6)]
    churn = []
    for k in range(12):                       # 12 learners in and out again
        churn += [(CC.ADD_LEARNER, 100 + k), (CC.REMOVE_NODE, 100 + k)]
    plans.append(churn + [(CC.ADD_LEARNER, 200)])
    # 6 members + 19 new learners alive at once: past the 24-entry table
    plans.append([(CC.ADD_LEARNER, 300 + k) for k in range(19)])
    for step, ccs in enumerate(plans):
        table, err, err_id = table.change([1] * G, [ccs] * G, [50 + step] * G)
        dev = CP.unpack(table.numpy(), 4)
        for g in range(G):
            nt, e = CP.oracle_apply(orc[g], 1, ccs, 50 + step)
            got_e = error_text(int(err[g]), int(err_id[g])) if err[g] else None
            if step < len(plans) - 1:
                assert got_e == e is None, (step, got_e, e)
                assert _render(dev[g]) == _render(nt), step
                orc[g] = nt
            else:   # the reference accepts 25 members; the engine reports its limit
                assert e is None and got_e is not None and "engine limit" in got_e


def test_restore_batch():
    from etcd_amd.quorum.confchange import restore
    r = random.Random(11)
    G = 300
    states = []
    for _ in range(G):
        ids = list(range(1, 1 + r.randint(1, 10)))
        r.shuffle(ids)
        nv = r.randint(1, len(ids))
        voters, rest = ids[:nv], ids[nv:]
        nl = r.randint(0, len(rest))
        learners = rest[:nl]
        outgoing, lnext = [], []
        if r.random() < 0.5:
            pool = voters + rest[nl:]
            outgoing = r.sample(pool, r.randint(1, len(pool)))
            cand = [i for i in outgoing if i not in voters]
            lnext = r.sample(cand, r.randint(0, len(cand)))
            learners = [i for i in learners if i not in outgoing]
        states.append(dict(voters=voters, learners=learners, voters_outgoing=outgoing,
                           learners_next=lnext, auto_leave=bool(outgoing) and r.random() < 0.5))
    table, err, _ = restore(_table([CC.Tracker.empty(5) for _ in range(G)], K=5), states,
                            [10] * G)
    assert not err.any()
    dev = CP.unpack(table.numpy(), 5)
    for g, cs in enumerate(states):
        want = CC.restore(CC.Tracker.empty(5), 10, cs["voters"], cs["learners"],
                          cs["voters_outgoing"], cs["learners_next"], cs["auto_leave"])
        assert _render(dev[g]) == _render(want), g


def test_quick_simple_equals_joint_on_device():
    """confchange/quick_test.go:30-144 batch-wide: every group's changes applied
    as a chain of Simple calls and as EnterJoint + LeaveJoint give the same
    config and Progress on the device (and match the oracle)."""
    from tests.test_confchange_oracle import _quick_inputs, _simple_chain
    r = random.Random(9)
    G = 1500
    inputs = [_quick_inputs(r) for _ in range(G)]
    base = [_simple_chain(CC.Tracker.empty(10), s) for s, _ in inputs]
    t1 = _table(base)
    steps = max(len(c) for _, c in inputs)
    for k in range(steps):
        op = [1 if k < len(c) else 0 for _, c in inputs]
        ccs = [[c[k]] if k < len(c) else [] for _, c in inputs]
        t1, err, _ = t1.change(op, ccs, [10] * G)
        assert not err.any()
    for al_op in (2, 3):
        j, err, _ = _table(base).change([al_op] * G, [c for _, c in inputs], [10] * G)
        assert not err.any()
        t2, err, _ = j.change([4] * G, [[] for _ in range(G)], [10] * G)
        assert not err.any()
        a, b = CP.unpack(t1.numpy(), 10), CP.unpack(t2.numpy(), 10)
        for g in range(G):
            assert _render(a[g]) == _render(b[g]), g
    want = [_render(_simple_chain(base[g], inputs[g][1])) for g in range(G)]
    assert [_render(x) for x in CP.unpack(t1.numpy(), 10)] == want


@pytest.mark.parametrize("short", [1, 7, 0.5])
def test_short_capacity_writes_nothing_past_it(short):
    """qb_dev_conf_change with slot_cap below new_off[G] (include/
    quorum_batch.h: nothing past the capacity is written): new_off, err and
    cfg equal a full-capacity call's, every group that fits is placed exactly
    (IDs, Progress rows, rings), and no per-slot entry at or past slot_cap
    changes (the outputs are sentinel-filled)."""
    import torch
    from etcd_amd import _lib
    r = random.Random(21)
    G, K = 700, 4
    orc = [CC.Tracker.empty(K) for _ in range(G)]
    table = _table(orc, K=K)
    for _ in range(2):  # a populated start
        op = [CP.random_op(r, t) for t in orc]
        ccs = [CP.random_ccs(r) for _ in orc]
        last = [r.randint(0, 1000) for _ in orc]
        table, _, _ = table.change(op, ccs, last)
        orc = [CP.oracle_apply(t, o_, c, l)[0] for t, o_, c, l in zip(orc, op, ccs, last)]
    op = [CP.random_op(r, t) for t in orc]
    ccs = [CP.random_ccs(r) for _ in orc]
    last = [r.randint(0, 1000) for _ in orc]
    full, err_f, _ = table.change(op, ccs, last)
    ref = full.numpy()
    S_new = int(ref["off"][G])
    cap = max(1, int(S_new * short)) if isinstance(short, float) else S_new - short
    dev = table.t["off"].device
    sent = {"ids": -7, "match": -7, "next": -7, "pending_snapshot": -7, "pstate": 0xAB,
            "infl_pos": -7}
    pad = 64
    o = {"new_off": torch.zeros(G + 1, dtype=torch.int32, device=dev),
         "cfg": torch.empty(G, dtype=torch.int32, device=dev),
         "ext": torch.empty(G, dtype=torch.int32, device=dev),
         "err": torch.empty(G, dtype=torch.uint8, device=dev),
         "err_id": torch.empty(G, dtype=torch.int64, device=dev)}
    for k, dt in (("ids", torch.int64), ("match", torch.int64), ("next", torch.int64),
                  ("pending_snapshot", torch.int64), ("pstate", torch.uint8),
                  ("infl_pos", torch.int32)):
        o[k] = torch.full((cap + pad,), sent[k], dtype=dt, device=dev)
    o["infl_buf"] = torch.full(((cap + pad) * K,), -7, dtype=torch.int64, device=dev)
    o_cap = dict(o)  # views of the first cap entries: the call's capacity
    for k in sent:
        o_cap[k] = o[k][:cap]
    o_cap["infl_buf"] = o["infl_buf"][:cap * K]
    with pytest.raises(_lib.QuorumBatchError):
        table.change(op, ccs, last, out=o_cap)
    torch.cuda.synchronize()
    new_off = o["new_off"].cpu().numpy().view(np.uint32)
    assert np.array_equal(new_off, ref["off"].astype(np.uint32))
    assert np.array_equal(o["err"].cpu().numpy(), err_f)
    okg = [g for g in range(G) if not err_f[g]]
    assert np.array_equal(o["cfg"].cpu().numpy()[okg], ref["cfg"][okg])
    h = {k: o[k].cpu().numpy() for k in list(sent) + ["infl_buf"]}
    fits = 0
    for g in range(G):
        a, b = int(new_off[g]), int(new_off[g + 1])
        if b > cap:
            break
        fits += 1
        for k in sent:
            assert np.array_equal(h[k][a:b], np.asarray(ref[k][a:b]).astype(h[k].dtype)), (g, k)
        assert np.array_equal(h["infl_buf"][a * K:b * K],
                              np.asarray(ref["infl_buf"][a * K:b * K]).astype(np.int64)), g
    assert fits > 0
    for k in sent:
        assert (h[k][cap:] == np.array(sent[k]).astype(h[k].dtype)).all(), k
    assert (h["infl_buf"][cap * K:] == -7).all()


def _ring_marks(table, K):
    """Give every old slot a unique nonzero match marker and a ring of
    (marker, k) words; returns {marker: ring} (test-only identities)."""
    import torch
    from etcd_amd.quorum.confchange import ConfigTable
    a = table.numpy()
    S = int(a["off"][-1])
    marks = np.arange(1, S + 1, dtype=np.uint64) * np.uint64(1000)
    a["match"][:S] = marks
    ring = (marks[:, None] + np.arange(1, K + 1, dtype=np.uint64)[None, :]).reshape(-1)
    prog = {k: a[k] for k in ("match", "next", "pending_snapshot", "pstate", "infl_pos")}
    prog["infl_buf"] = ring if K else np.zeros(1, np.uint64)
    t = ConfigTable.from_numpy(a["off"], a["ids"], a["cfg"], a["ext"], prog, K)
    rings = {int(m): ring[i * K:(i + 1) * K] for i, m in enumerate(marks)}
    return t, rings


def _check_rings(new, rings, K):
    """A carried slot (its old match marker survives) keeps its old ring word
    for word; a fresh one (initProgress: match 0) has an empty one."""
    a = new.numpy()
    S = int(a["off"][-1])
    for s in range(S):
        got = a["infl_buf"][s * K:(s + 1) * K]
        m = int(a["match"][s])
        want = rings[m] if m in rings else np.zeros(K, np.uint64)
        assert np.array_equal(got, want), (s, m, got, want)


@pytest.mark.parametrize("K", [0, 1, 3, 4, 8])
def test_ring_sizes_vs_oracle(K):
    """k_cc_move's K == 4 / K < 4 / K > 4 ring branches (K = 0 with
    no ring at all) against the oracle's configs and Progress, and every
    carried ring moved word for word (fresh slots start empty)."""
    r = random.Random(40 + K)
    G = 900
    orc = [CC.Tracker.empty(K) for _ in range(G)]
    table = _table(orc, K=K)
    for step in range(6):
        op = [CP.random_op(r, t) for t in orc]
        ccs = [CP.random_ccs(r) for _ in orc]
        last = [r.randint(0, 1000) for _ in orc]
        marked, rings = _ring_marks(table, K)
        host = marked.numpy()      # the oracle carries the same markers
        for g in range(G):
            for s in range(int(host["off"][g]), int(host["off"][g + 1])):
                orc[g].prs[int(host["ids"][s])].match = int(host["match"][s])
        table, err, err_id = marked.change(op, ccs, last)
        dev = CP.unpack(table.numpy(), K)
        for g in range(G):
            nt, e = CP.oracle_apply(orc[g], op[g], ccs[g], last[g])
            if e is None and sum(1 for _ in nt.prs) > 16:
                nt, e = orc[g], "engine limit"
            assert bool(err[g]) == (e is not None), (K, step, g, e)
            assert _render(dev[g]) == _render(nt), (K, step, g)
            orc[g] = nt
        if K:
            _check_rings(table, rings, K)


def test_ring16_unaligned_buffers_take_the_word_loop():
    """inflight_cap 4 with ring buffers only 8-byte aligned (views
    one element into larger tensors) gives exactly the aligned call's
    result."""
    import torch
    r = random.Random(77)
    G, K = 700, 4
    orc = [CC.Tracker.empty(K) for _ in range(G)]
    table = _table(orc, K=K)
    for _ in range(2):
        op = [CP.random_op(r, t) for t in orc]
        ccs = [CP.random_ccs(r) for _ in orc]
        table, _, _ = table.change(op, ccs, [5] * G)
    table, rings = _ring_marks(table, K)
    op = [CP.random_op(r, t) for t in orc]
    ccs = [CP.random_ccs(r) for _ in orc]
    ref, err_ref, _ = table.change(op, ccs, [9] * G)
    dev = table.t["off"].device
    big = torch.zeros(table.t["infl_buf"].numel() + 1, dtype=torch.int64, device=dev)
    big[1:] = table.t["infl_buf"]
    table.t["infl_buf"] = big[1:]
    assert table.t["infl_buf"].data_ptr() % 16 == 8
    cap = int(ref.numpy()["off"][-1]) + 8
    o = {"new_off": torch.zeros(G + 1, dtype=torch.int32, device=dev),
         "cfg": torch.empty(G, dtype=torch.int32, device=dev),
         "ext": torch.empty(G, dtype=torch.int32, device=dev),
         "err": torch.empty(G, dtype=torch.uint8, device=dev),
         "err_id": torch.empty(G, dtype=torch.int64, device=dev),
         "ids": torch.empty(cap, dtype=torch.int64, device=dev),
         "match": torch.empty(cap, dtype=torch.int64, device=dev),
         "next": torch.empty(cap, dtype=torch.int64, device=dev),
         "pending_snapshot": torch.empty(cap, dtype=torch.int64, device=dev),
         "pstate": torch.empty(cap, dtype=torch.uint8, device=dev),
         "infl_pos": torch.empty(cap, dtype=torch.int32, device=dev)}
    ob = torch.zeros(cap * K + 1, dtype=torch.int64, device=dev)
    o["infl_buf"] = ob[1:]
    got, err, _ = table.change(op, ccs, [9] * G, out=o)
    assert np.array_equal(err, err_ref)
    a, b = got.numpy(), ref.numpy()
    for k in b:
        assert np.array_equal(a[k], b[k]), k
    _check_rings(got, rings, K)


@pytest.mark.parametrize("learners", [15, 25, 40])
def test_wide_wave_owner_lookup(learners):
    """a wave of 64 groups whose slots exceed k_cc_move's owner
    table (64 x QB_MAX_SLOTS): groups of 5 voters and 15 learners kept as they
    are (no operation) and refused (a learner more breaks the engine's
    16-member limit: the old slots stay) — every slot found by the binary
    search and moved exactly, rings included.  With 25 and 40 learners the
    groups exceed the replay's 24-entry working table too (and 40 the 32-bit
    role masks): they are never replayed, copied through or refused the same
    way."""
    K = 3
    G = 256
    ns = 5 + learners

    def tracker(g):
        prs = {i: CC.Pr(match=0, next=10 + g, inflight_size=K) for i in range(1, 6)}
        prs.update({i: CC.Pr(match=0, next=20 + g, is_learner=True, inflight_size=K)
                    for i in range(100, 100 + learners)})
        return CC.Tracker(set(range(1, 6)), None, set(range(100, 100 + learners)), None, False,
                          prs, K)
    import torch
    orc = [tracker(g) for g in range(G)]
    table, rings = _ring_marks(_table(orc, K=K), K)
    before = table.numpy()
    dev = table.t["off"].device
    cap = ns * G + 8   # (the default capacity assumes <= 16 slots per group)
    for op, ccs in ((0, []), (1, [(CC.ADD_LEARNER, 200)])):
        o = {"new_off": torch.zeros(G + 1, dtype=torch.int32, device=dev),
             "cfg": torch.empty(G, dtype=torch.int32, device=dev),
             "ext": torch.empty(G, dtype=torch.int32, device=dev),
             "err": torch.empty(G, dtype=torch.uint8, device=dev),
             "err_id": torch.empty(G, dtype=torch.int64, device=dev),
             "pstate": torch.empty(cap, dtype=torch.uint8, device=dev),
             "infl_pos": torch.empty(cap, dtype=torch.int32, device=dev),
             "infl_buf": torch.empty(cap * K, dtype=torch.int64, device=dev)}
        for k in ("ids", "match", "next", "pending_snapshot"):
            o[k] = torch.empty(cap, dtype=torch.int64, device=dev)
        got, err, _ = table.change([op] * G, [ccs] * G, [50] * G, out=o)
        a = got.numpy()
        assert int(a["off"][-1]) == ns * G
        assert (err == (15 if op else 0)).all()
        for k in ("off", "ids", "cfg", "match", "next", "pstate"):
            assert np.array_equal(a[k], before[k]), (op, k)
        _check_rings(got, rings, K)


def test_out_validation_refuses_bad_buffers():
    """change(out=...) refuses, before any device write, an output
    set with a short per-slot array or ring, a missing key, a host tensor, a
    wrong element size, a non-contiguous view, or a buffer aliasing the
    input table."""
    import torch
    from etcd_amd import _lib
    r = random.Random(5)
    G, K = 300, 4
    orc = [CC.Tracker.empty(K) for _ in range(G)]
    table = _table(orc, K=K)
    op = [CP.random_op(r, t) for t in orc]
    ccs = [CP.random_ccs(r) for _ in orc]
    dev = table.t["off"].device
    cap = 4 * G

    def good():
        o = {"new_off": torch.zeros(G + 1, dtype=torch.int32, device=dev),
             "cfg": torch.empty(G, dtype=torch.int32, device=dev),
             "ext": torch.empty(G, dtype=torch.int32, device=dev),
             "err": torch.empty(G, dtype=torch.uint8, device=dev),
             "err_id": torch.empty(G, dtype=torch.int64, device=dev),
             "pstate": torch.empty(cap, dtype=torch.uint8, device=dev),
             "infl_pos": torch.empty(cap, dtype=torch.int32, device=dev),
             "infl_buf": torch.empty(cap * K, dtype=torch.int64, device=dev)}
        for k in ("ids", "match", "next", "pending_snapshot"):
            o[k] = torch.empty(cap, dtype=torch.int64, device=dev)
        return o
    table.change(op, ccs, [3] * G, out=good())          # accepted
    bad = []
    o = good(); o["infl_buf"] = o["infl_buf"][: cap * K - 1]; bad.append(o)
    bad.append(good()); del bad[-1]["err_id"]
    o = good(); o["cfg"] = o["cfg"].cpu(); bad.append(o)
    o = good(); o["infl_pos"] = o["infl_pos"].to(torch.int64); bad.append(o)
    o = good(); o["ids"] = torch.empty(2 * cap, dtype=torch.int64, device=dev)[::2]; bad.append(o)
    o = good(); o["match"] = table.t["match"]; bad.append(o)
    o = good(); o["next"] = o["ids"]; bad.append(o)
    o = good(); o["new_off"] = o["new_off"][:G]; bad.append(o)
    for o in bad:
        with pytest.raises(_lib.QuorumBatchError):
            table.change(op, ccs, [3] * G, out=o)
    # a shorter per-slot array sets the capacity: nothing past it is written
    o = good()
    o["match"] = torch.full((40,), -7, dtype=torch.int64, device=dev)
    with pytest.raises(_lib.QuorumBatchError, match="capacity 40"):
        table.change(op, ccs, [3] * G, out=o)
    assert int(o["new_off"][G].item()) > 40
