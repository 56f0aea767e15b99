"""The leader-step oracle (oracle/leader_ref.py) against the reference's own
tests for this path, transcribed in tests/golden/leader_tables.json."""
import pytest

from oracle import leader_ref as L
from tests import leader_scenarios as LS

TABLES = LS.load_tables()


@pytest.mark.parametrize("sc", TABLES["scenarios"], ids=[s["name"] for s in TABLES["scenarios"]])
def test_scenario(sc):
    LS.run_scenario_oracle(sc)


def test_progress_is_paused():
    for state, paused, want in TABLES["progress"]["TestProgressIsPaused"]:
        p = L.Progress(state=state, probe_sent=paused)
        assert p.is_paused() == want


def test_progress_become_probe():
    for state, nxt, psnap, wnext in TABLES["progress"]["TestProgressBecomeProbe"]:
        p = L.Progress(state=state, match=1, next=nxt, pending_snapshot=psnap)
        p.become_probe()
        assert (p.state, p.match, p.next) == (L.STATE_PROBE, 1, wnext)


def test_progress_become_replicate_snapshot():
    t = TABLES["progress"]["TestProgressBecomeReplicate"]
    p = L.Progress(state=L.STATE_PROBE, match=t["match"], next=t["next"])
    p.become_replicate()
    assert (p.state, p.match, p.next) == (L.STATE_REPLICATE, t["match"], t["wnext"])
    t = TABLES["progress"]["TestProgressBecomeSnapshot"]
    p = L.Progress(state=L.STATE_PROBE, match=t["match"], next=t["next"])
    p.become_snapshot(t["snap"])
    assert (p.state, p.match, p.pending_snapshot) == (L.STATE_SNAPSHOT, t["match"], t["snap"])


def test_progress_maybe_decr():
    for state, m, n, rejected, last, w, wn in TABLES["progress"]["TestProgressMaybeDecr"]:
        p = L.Progress(state=state, match=m, next=n)
        assert p.maybe_decr_to(rejected, last) == w
        assert (p.match, p.next) == (m, wn)


def test_progress_resume():
    t = TABLES["progress"]["TestProgressResume"]
    p = L.Progress(next=t["next"], probe_sent=True)
    p.maybe_decr_to(*t["decr"])
    assert not p.probe_sent
    p.probe_sent = True
    p.maybe_update(t["update"])
    assert not p.probe_sent


@pytest.mark.parametrize("case", TABLES["inflights"], ids=[c["name"] for c in TABLES["inflights"]])
def test_inflights(case):
    infl = L.Inflights(case["size"], start=case["start"])
    for op in case["ops"]:
        if op[0] == "add":
            for v in op[1]:
                infl.add(v)
        elif op[0] == "free_le":
            infl.free_le(op[1])
        elif op[0] == "free_first_one":
            infl.free_first_one()
        else:
            _, start, count, buf = op
            assert (infl.start, infl.count, infl.buffer) == (start, count, buf)


def test_pack_round_trip():
    import copy
    import numpy as np
    from tests import leader_pack as LP
    rng = np.random.default_rng(3)
    gs = LP.random_groups(rng, 200, 4, 3, max_slots=16)
    a = LP.pack(gs, 4, 3)
    g2 = copy.deepcopy(gs)
    for g in g2:
        for p in g.prs:
            p.match += 1
    LP.unpack_into(g2, a, 4, 3)
    assert [LP.state_key(g) for g in gs] == [LP.state_key(g) for g in g2]


def test_find_conflict_by_term_matches_linear_walk():
    """The engine walks term runs; the oracle restates log.go:150-171 index by
    index.  Both must agree on every (index, term) of random logs."""
    import numpy as np
    rng = np.random.default_rng(9)
    for _ in range(300):
        first = int(rng.integers(1, 10))
        last = first - 1 + int(rng.integers(0, 30))
        starts = sorted(set([first - 1] + [int(x) for x in rng.integers(first - 1, last + 2, 4)]))
        terms = sorted(int(x) for x in rng.integers(0, 9, len(starts)))
        log = L.LogView(first, last, 0, list(zip(starts, terms)))
        for idx in range(0, last + 3):
            for t in range(0, 10):
                got = log.find_conflict_by_term(idx, t)
                # run-jumping form (qb_leader.hip find_conflict_by_term)
                i = idx
                if i <= last:
                    while True:
                        if i < first - 1 or i > last:
                            break
                        rt, rs = 0, 0
                        for s, tt in log.runs:
                            if s <= i:
                                rt, rs = tt, s
                        if rt <= t:
                            break
                        i = (max(rs, first - 1) - 1) & L.M64
                assert got == i


def _records_soa(recs):
    import numpy as np
    from tests import leader_pack as LP
    a = LP.records_arrays(recs)
    flags = (a["slot"] & 0x0F) | ((a["kind"] & 3) << 4) | (a["reject"].astype(np.uint8) << 7)
    return {"group": a["group"], "flags": flags.astype(np.uint8), "index": a["index"],
            "term": a["term"], "hint": a["hint"], "log_term": a["log_term"]}


@pytest.mark.parametrize("seed,read_only,threads", [(1, 0, 1), (2, 1, 1), (3, 0, 4)])
def test_c_oracle_matches_python_oracle(seed, read_only, threads):
    """The full-size checker (oracle/leader_oracle.c) against the pinned
    Python restatement on random leader states and batches."""
    import copy
    import numpy as np
    from tests import leader_pack as LP
    from tests import oracle_c as oc
    rng = np.random.default_rng(seed)
    gs = LP.random_groups(rng, 600, 3, 4, max_slots=16 if read_only else 9)
    for g in gs:
        g.read_only = read_only
    recs = LP.random_records(rng, gs, 2000)
    arrays = LP.pack(gs, 3, 4)
    msgs, total, sd, gf, stats = oc.leader_step(arrays, 3, 4, read_only, _records_soa(recs),
                                                threads=threads)
    orc = copy.deepcopy(gs)
    for g in orc:
        g.msgs = []
    st = L.run_batch(orc, recs)
    dev = copy.deepcopy(gs)
    LP.unpack_into(dev, arrays, 3, 4)
    assert [LP.state_key(g) for g in dev] == [LP.state_key(g) for g in orc]
    want = [(gi,) + m.key() for gi, g in enumerate(orc) for m in g.msgs]
    got = [(int(m["group"]), int(m["type"]), int(m["to"]), int(m["index"]), int(m["log_term"]),
            int(m["commit"]), int(m["aux"])) for m in msgs]
    assert total == len(want) and got == want
    assert [int(x) for x in stats[:6]] == [st["applied"], st["stale"], st["higher"],
                                           st["nonmember"], st["after"], st["bad"]]
    want_sd = [0xFFFFFFFF if g.stepped_down_at is None else g.stepped_down_at for g in orc]
    assert sd.tolist() == want_sd
    want_fl = [(1 if g.advanced else 0) | (2 if g.released_pending else 0)
               | (4 if g.stepped_down_at is not None else 0) for g in orc]
    assert gf.tolist() == want_fl
