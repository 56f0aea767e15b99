"""The raftpb wire restatement (oracle/raftpb_ref.py) against Google's
protobuf runtime — an independent implementation of the same wire format —
on a descriptor built from raft.proto:68-86 (Message), Entry, Snapshot,
SnapshotMetadata and ConfState, plus every error path of the generated Go
Unmarshal (raft.pb.go) on hand-built malformed inputs."""
import random

import pytest

from oracle import raftpb_ref as W


def _pool():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name="raftpb_test.proto", package="raftpb",
                                            syntax="proto2")
    F = descriptor_pb2.FieldDescriptorProto
    U64, BOOL, BYTES, MSG = F.TYPE_UINT64, F.TYPE_BOOL, F.TYPE_BYTES, F.TYPE_MESSAGE
    OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, lab, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=lab)
            if tname:
                f.type_name = ".raftpb." + tname
    # enum-typed fields are declared uint64 here: same varint wire encoding
    msg("ConfState", [("voters", 1, U64, REP, None), ("learners", 2, U64, REP, None),
                      ("voters_outgoing", 3, U64, REP, None), ("learners_next", 4, U64, REP, None),
                      ("auto_leave", 5, BOOL, OPT, None)])
    msg("SnapshotMetadata", [("conf_state", 1, MSG, OPT, "ConfState"), ("index", 2, U64, OPT, None),
                             ("term", 3, U64, OPT, None)])
    msg("Snapshot", [("data", 1, BYTES, OPT, None), ("metadata", 2, MSG, OPT, "SnapshotMetadata")])
    msg("Entry", [("Type", 1, U64, OPT, None), ("Term", 2, U64, OPT, None),
                  ("Index", 3, U64, OPT, None), ("Data", 4, BYTES, OPT, None)])
    msg("Message", [("type", 1, U64, OPT, None), ("to", 2, U64, OPT, None),
                    ("from", 3, U64, OPT, None), ("term", 4, U64, OPT, None),
                    ("logTerm", 5, U64, OPT, None), ("index", 6, U64, OPT, None),
                    ("entries", 7, MSG, REP, "Entry"), ("commit", 8, U64, OPT, None),
                    ("snapshot", 9, MSG, OPT, "Snapshot"), ("reject", 10, BOOL, OPT, None),
                    ("rejectHint", 11, U64, OPT, None), ("context", 12, BYTES, OPT, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName("raftpb." + n)) for n in
            ("Message", "Entry", "Snapshot", "SnapshotMetadata", "ConfState")}


try:
    P = _pool()
except Exception as e:  # pragma: no cover
    P = None
    _why = str(e)

needs_pb = pytest.mark.skipif(P is None, reason="google.protobuf unavailable")


def _rand_u64(r):
    return r.choice([0, 1, 127, 128, 300, (1 << 32) - 1, 1 << 32, (1 << 63) - 1, 1 << 63,
                     (1 << 64) - 1, r.getrandbits(64), r.getrandbits(20)])


def _google_message(r):
    m = P["Message"]()
    vals = dict(type=r.choice([4, 9, 10, 11, 3, 6, 18]), to=_rand_u64(r), frm=_rand_u64(r),
                term=_rand_u64(r), log_term=_rand_u64(r), index=_rand_u64(r),
                commit=_rand_u64(r), reject=r.random() < 0.5, reject_hint=_rand_u64(r))
    m.type, m.to, m.term, m.logTerm, m.index = (vals["type"], vals["to"], vals["term"],
                                                vals["log_term"], vals["index"])
    setattr(m, "from", vals["frm"])
    m.commit, m.reject, m.rejectHint = vals["commit"], vals["reject"], vals["reject_hint"]
    ents = []
    for _ in range(r.randint(0, 2)):
        e = m.entries.add()
        e.Type, e.Term, e.Index = r.randint(0, 2), _rand_u64(r), _rand_u64(r)
        e.Data = bytes(r.getrandbits(8) for _ in range(r.randint(0, 5)))
        ents.append(W.marshal_entry(e.Term, e.Index, e.Type, e.Data))
    cs = m.snapshot.metadata.conf_state
    voters = [_rand_u64(r) for _ in range(r.randint(0, 3))]
    cs.voters.extend(voters)
    cs.auto_leave = False
    m.snapshot.metadata.index = 0
    m.snapshot.metadata.term = 0
    ctx = None
    if r.random() < 0.5:
        ctx = bytes(r.getrandbits(8) for _ in range(r.choice([0, 8, 3])))
        m.context = ctx
    mine = W.marshal_message(vals["type"], vals["to"], vals["frm"], vals["term"],
                             vals["log_term"], vals["index"], ents, vals["commit"],
                             W.marshal_snapshot(conf_state=W.marshal_conf_state(voters)),
                             vals["reject"], vals["reject_hint"], ctx)
    return m, mine, vals, ctx


@needs_pb
def test_encoder_matches_google_protobuf():
    r = random.Random(7)
    for _ in range(500):
        m, mine, _, _ = _google_message(r)
        assert m.SerializeToString() == mine


@needs_pb
def test_decoder_matches_google_protobuf_on_valid_input():
    r = random.Random(8)
    for _ in range(500):
        m, mine, vals, ctx = _google_message(r)
        ok, f = W.decode_message(mine)
        assert ok
        back = P["Message"]()
        back.ParseFromString(mine)
        assert f[1] == back.type and f[2] == back.to and f[3] == getattr(back, "from")
        assert (f[4], f[5], f[6], f[8], f[11]) == (back.term, back.logTerm, back.index,
                                                    back.commit, back.rejectHint)
        assert bool(f[10]) == back.reject
        assert f.get(12) == (ctx if ctx is not None else None)
        assert len(f.get(7, [])) == len(back.entries)


@needs_pb
def test_decoder_accepts_google_variants():
    """Field order, packed repeated, omitted defaults and unknown fields are
    all valid wire forms the reference decodes."""
    r = random.Random(9)
    for _ in range(200):
        m, _, _, _ = _google_message(r)
        raw = m.SerializeToString()
        # unknown field 99 (varint), 100 (fixed64), 101 (bytes)
        extra = W._key(99, 0) + W.varint(5) + W._key(100, 1) + b"\x01" * 8 + W._key(101, 2) + b"\x02ab"
        ok, f = W.decode_message(extra + raw + extra)
        assert ok and f[6] == m.index
    cs = P["ConfState"]()
    cs.voters.extend([1, 300, 1 << 40])
    packed = W._key(1, 2) + W.varint(len(W.varint(1) + W.varint(300) + W.varint(1 << 40))) + \
        W.varint(1) + W.varint(300) + W.varint(1 << 40)
    assert W.unmarshal("ConfState", packed)[1] == [1, 300, 1 << 40]
    back = P["ConfState"]()
    back.ParseFromString(packed)
    assert list(back.voters) == [1, 300, 1 << 40]


def test_error_paths():
    ok = lambda b: W.decode_message(b)[0]
    good = W.marshal_message(4, 1, 2, 3, 0, 5)
    assert ok(good) and ok(b"")
    assert not ok(good[:-1])                                   # truncated varint / field
    assert not ok(b"\x08" + b"\xff" * 10 + b"\x01")             # varint overflow
    assert ok(b"\x08" + b"\xff" * 9 + b"\x01")                  # 10-byte varint is fine
    assert not ok(b"\x0c")                                      # wiretype 4 at field level
    assert not ok(b"\x00\x00")                                  # field number 0
    assert not ok(b"\x0a\x00")                                  # type with wiretype 2
    assert not ok(b"\x62\x05abc")                               # context longer than input
    assert not ok(b"\x62" + W.varint((1 << 64) - 1))           # negative length
    assert not ok(b"\x3a\x02\x12\x01")                          # entry: wrong wiretype inside
    assert not ok(b"\x4a\x02\x08\x00")                          # snapshot field 1 must be bytes
    assert ok(W._key(50, 3) + W._key(51, 0) + b"\x01" + W._key(50, 4))   # skipped group
    assert not ok(W._key(50, 3) + W._key(51, 0) + b"\x01")      # unterminated group
    assert not ok(W._key(50, 6))                                 # illegal wiretype
    assert not ok(W._key(50, 1) + b"\x00" * 7)                  # fixed64 past the end
    # field number int32(key >> 3) == 1 for a key with bit 35 set
    assert W.decode_message(W.varint(((1 << 32) + 1) << 3) + b"\x04")[1][1] == 4
    # packed ConfState element runs past the packed length but inside the slice
    cs = W._key(1, 2) + b"\x01" + b"\x81\x01"
    assert W.unmarshal("ConfState", cs) == {1: [129]}


def test_ingest_contract():
    ids = [3, 7, 9]
    st = W.ingest(W.marshal_message(4, 3, 7, 5, 0, 42, reject=True, reject_hint=40), 11, ids)
    assert st == (W.ST_OK, 11, 1 | 0x80, 42, 5, 40, 0, 4)
    st = W.ingest(W.marshal_message(9, 3, 8, 5, context=(12345).to_bytes(8, "big")), 11, ids)
    assert st == (W.ST_OK, 11, W.NO_PROGRESS | 0x10, 12345, 5, 0, 0, 9)
    assert W.ingest(W.marshal_message(9, 3, 9, 5, context=b"abc"), 11, ids)[0] == W.ST_CTX
    assert W.ingest(W.marshal_message(6, 3, 9, 5), 11, ids)[0] == W.ST_TYPE
    assert W.ingest(b"\x00", 11, ids)[0] == W.ST_UNMARSHAL


def test_c_ingest_matches_python_restatement():
    import numpy as np
    from tests import oracle_c as oc
    from tests.wire_gen import groups_ids, random_message
    r = random.Random(3)
    G = 200
    off, ids = groups_ids(r, G)
    msgs, groups = [], []
    for _ in range(5000):
        g = r.randrange(G + 2)
        msgs.append(random_message(r, ids[off[g]:off[g + 1]].tolist() if g < G else []))
        groups.append(g)
    moff = np.zeros(len(msgs) + 1, np.uint64)
    moff[1:] = np.cumsum([len(m) for m in msgs])
    buf = np.frombuffer(b"".join(msgs), np.uint8).copy()
    out = oc.ingest(buf, moff, np.array(groups, np.uint32), off, ids, threads=3)
    for i, (b, g) in enumerate(zip(msgs, groups)):
        want = W.ingest(b, g, ids[off[g]:off[g + 1]].tolist() if g < G else [])
        got = (int(out["status"][i]), int(out["group"][i]), int(out["flags"][i]),
               int(out["index"][i]), int(out["term"][i]), int(out["hint"][i]),
               int(out["log_term"][i]))
        assert got == tuple(want[:7]), (i, b.hex())


def _crc32c(data: bytes) -> int:
    """CRC-32 with the Castagnoli polynomial (reflected 0x82F63B78), as Go's
    crc32.MakeTable(crc32.Castagnoli) + crc32.Checksum."""
    crc = 0xFFFFFFFF
    for byte in data:
        crc ^= byte
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def test_wire_primitives_pinned_by_reference_bytes(monkeypatch):
    """The only protobuf-encoded bytes the reference holds as a fixture are a
    walpb.Record (server/storage/wal/record_test.go:29-30, decoded by the
    test to Record{Type: 1, Crc: crc32c(infoData), Data: infoData}, :43).
    walpb is gogoproto like raftpb, so this pins the restated decoder's
    primitives — multi-byte varints and length-delimited fields — on
    reference-held bytes; no reference fixture holds raftpb.Message bytes, so
    Message-level wire parity stays unpinned."""
    from oracle import raftpb_ref as R
    monkeypatch.setitem(R.SCHEMAS, "walpb.Record", {1: "v", 2: "v", 3: "b"})
    info = b"\b\xef\xfd\x02"
    record = b"\x0e\x00\x00\x00\x00\x00\x00\x00\b\x01\x10\x99\xb5\xe4\xd0\x03\x1a\x04" + info
    body = record[8:]            # the 8-byte frame length precedes the protobuf (decoder.go)
    got = R.unmarshal("walpb.Record", body)
    assert got == {1: 1, 2: _crc32c(info), 3: info}
    # truncations the reference test expects to fail with io.ErrUnexpectedEOF (:46-47)
    for cut in (len(body) - len(info), len(body) - 1):
        with pytest.raises(R.WireError):
            R.unmarshal("walpb.Record", body[:cut])


def _fixture_schema():
    import json
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "raftpb_schema.json")
    with open(path) as f:
        d = json.load(f)
    return {k: {int(n): v for n, v in fs.items()} for k, fs in d["messages"].items()}


def test_schemas_pinned_by_reference_descriptor():
    """SCHEMAS (field numbers, wire types, embedded kinds) equals the schema
    decoded from the reference's own FileDescriptorProto bytes
    (raft.pb.go:698; tests/golden/raftpb_schema.json).  Message-value parity
    stays unpinned: the reference holds no encoded raftpb.Message."""
    from oracle import raftpb_ref as r
    fields = _fixture_schema()
    assert r.schema_from_descriptor(fields) == r.SCHEMAS


def test_fast_prefix_assumptions_pinned_by_reference_descriptor():
    """What the wire kernel's fast prefix (qb_wire.hip)
    relies on, read from the reference's descriptor: every Message field but
    context is non-nullable (gogoproto always writes it, in field order), as
    are Snapshot.metadata, SnapshotMetadata.conf_state and its index / term,
    Entry's Term / Index / Type; ConfState's repeated ids are unpacked
    (proto2) and auto_leave is non-nullable."""
    f = _fixture_schema()
    msg = f["Message"]
    assert [n for n in sorted(msg) if msg[n]["nullable"]] == [12]        # context
    assert msg[7]["label"] == 3 and msg[9]["label"] == 1                 # entries repeated
    assert not f["Snapshot"][2]["nullable"] and f["Snapshot"][1]["nullable"]
    assert not any(f["SnapshotMetadata"][n]["nullable"] for n in (1, 2, 3))
    assert not any(f["Entry"][n]["nullable"] for n in (1, 2, 3))
    cs = f["ConfState"]
    assert all(cs[n]["label"] == 3 and not cs[n]["packed"] for n in (1, 2, 3, 4))
    assert not cs[5]["nullable"]


def test_descriptor_fixture_regenerates_from_reference():
    """Where /root/reference is present (the build container), decoding its
    descriptor blob with the restated decoder reproduces the fixture, and
    Google's runtime agrees field by field (make_raftpb_schema.cross_check)."""
    import os
    if not os.path.exists("/root/reference/raft/raftpb/raft.pb.go"):
        pytest.skip("reference not present (GPU box)")
    from tests.golden import make_raftpb_schema as mk
    fdp = mk.reference_descriptor("/root/reference")
    schema = mk.decoded_schema(fdp)
    mk.cross_check(fdp, schema)
    assert {k: {int(n): v for n, v in fs.items()} for k, fs in schema.items()} == _fixture_schema()


def test_device_side_appresp_encoder_matches_marshal():
    """wire.encode_appresp (the composed wire -> tracker workload's generator,
    run here on CPU tensors) writes exactly the bytes the raftpb restatement's
    Marshal writes for the same MsgAppResp (which test_encoder_matches_google_
    protobuf pins to Google's runtime), and the C ingest decodes them back to
    the columns they came from; out-of-range fields are refused."""
    import numpy as np
    import torch
    from etcd_amd.quorum import wire
    from tests import oracle_c as oc
    rng = np.random.default_rng(3)
    M, G = 300, 50
    ids = (16384 + np.arange(5)[None, :] * 200000 + (np.arange(G) % 100000)[:, None]).reshape(-1)
    grp = rng.integers(0, G, M)
    slot = rng.integers(1, 5, M)
    to = torch.from_numpy(ids[grp * 5].astype(np.int64))
    frm = torch.from_numpy(ids[grp * 5 + slot].astype(np.int64))
    term = torch.from_numpy(rng.integers(1 << 14, 1 << 21, M).astype(np.int64))
    index = torch.from_numpy(rng.integers(1 << 35, 1 << 42, M).astype(np.int64))
    rej = torch.from_numpy(rng.random(M) < 0.3)
    buf, nb, moff = wire.encode_appresp(to, frm, term, index, rej)
    b = buf.numpy().tobytes()
    for i in range(M):
        want = W.marshal_message(4, int(to[i]), int(frm[i]), int(term[i]), 0, int(index[i]),
                                 reject=bool(rej[i]))
        assert b[int(moff[i]):int(moff[i + 1])] == want, i
    off = (np.arange(G + 1) * 5).astype(np.uint32)
    got = oc.ingest(buf.numpy(), moff.numpy().view(np.uint64), grp.astype(np.uint32), off,
                    ids.astype(np.uint64))
    assert (got["status"] == 0).all()
    assert np.array_equal(got["flags"], (slot | (rej.numpy().astype(np.int64) << 7)).astype(np.uint8))
    assert np.array_equal(got["index"], index.numpy().view(np.uint64))
    assert np.array_equal(got["term"], term.numpy().view(np.uint64))
    with pytest.raises(ValueError):
        wire.encode_appresp(to, frm, term, index - (1 << 35), rej)
