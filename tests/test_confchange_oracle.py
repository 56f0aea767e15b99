"""The confchange restatement (oracle/confchange_ref.py) against the
reference's datadriven testdata (tests/golden/confchange_datadriven.json) and
its Restore round-trip property (confchange/restore_test.go)."""
import json
import os
import random

import pytest

from oracle import confchange_ref as CC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DD = json.load(open(os.path.join(ROOT, "tests", "golden", "confchange_datadriven.json")))


@pytest.mark.parametrize("name", sorted(DD))
def test_datadriven(name):
    cases = DD[name]
    outs = CC.run_datadriven(cases)
    for c, got in zip(cases, outs):
        assert got == c["expected"], f"{name}:{c['line']}\n{got}\nwant\n{c['expected']}"


def test_restore_round_trip():
    """restore_test.go:87-142: Restore(ConfState) reproduces the ConfState
    (voters, learners, outgoing, learners_next, autoleave)."""
    r = random.Random(4)
    for _ in range(300):
        ids = list(range(1, 1 + r.randint(1, 12)))
        r.shuffle(ids)
        nv = r.randint(1, len(ids))
        voters = ids[:nv]
        rest = ids[nv:]
        nl = r.randint(0, len(rest))
        learners = rest[:nl]
        outgoing, lnext = [], []
        if r.random() < 0.5:
            pool = voters + rest[nl:]
            outgoing = r.sample(pool, r.randint(1, len(pool)))
            cand = [i for i in outgoing if i not in voters]
            lnext = r.sample(cand, r.randint(0, len(cand)))
            learners = [i for i in learners if i not in outgoing]
        auto = bool(outgoing) and r.random() < 0.5
        t = CC.restore(CC.Tracker.empty(20), 10, voters, learners, outgoing, lnext, auto)
        assert t.voters_in == set(voters)
        assert (t.voters_out or set()) == set(outgoing)
        assert (t.learners or set()) == set(learners)
        assert (t.learners_next or set()) == set(lnext)
        assert t.auto_leave == auto


def _quick_inputs(r):
    """confchange/quick_test.go:146-191 generators: setup = AddNode(1) + 1..5
    AddNode of IDs 1..5; changes = 1..9 of any type on IDs 2..10."""
    setup = [(CC.ADD_NODE, 1)] + [(CC.ADD_NODE, 1 + r.randrange(5))
                                  for _ in range(1 + r.randrange(5))]
    ccs = [(r.randrange(4), 2 + r.randrange(9)) for _ in range(1 + r.randrange(9))]
    return setup, ccs


def _simple_chain(t, ccs):
    for cc in ccs:
        t = CC.Changer(t, 10).simple([cc])
    return t


def test_quick_simple_equals_joint():
    """confchange/quick_test.go:30-144: applying changes one Simple at a time
    equals EnterJoint(ccs) + LeaveJoint (autoLeave either way)."""
    r = random.Random(5)
    for _ in range(2000):
        setup, ccs = _quick_inputs(r)
        base = _simple_chain(CC.Tracker.empty(10), setup)
        t1 = _simple_chain(base, ccs)
        for al in (False, True):
            j = CC.Changer(base, 10).enter_joint(al, ccs)
            t2 = CC.Changer(j, 10).leave_joint()
            assert t1.config_string() == t2.config_string()
            assert t1.progress_string() == t2.progress_string()
