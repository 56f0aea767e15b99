"""CPU restatement of raftpb's Message wire format — TEST INFRASTRUCTURE ONLY.

Checker for the wire-ingest kernel.  Only tests/ and
bench tooling import it.  Paths relative to the reference's raft/raftpb/:

  Message.Unmarshal           raft.pb.go:1739-2061
  Entry.Unmarshal             raft.pb.go:1360-1500
  SnapshotMetadata.Unmarshal  raft.pb.go:1501-1621
  Snapshot.Unmarshal          raft.pb.go:1622-1738
  ConfState.Unmarshal         raft.pb.go:2169-2542 (packed and unpacked
                              repeated uint64; a packed element's varint is
                              bounded by the enclosing slice, not the packed
                              length — restated as written)
  skipRaft                    raft.pb.go:2909-2988
  Message.MarshalToSizedBuffer raft.pb.go:903-972 (gogoproto non-nullable
                              fields are always written, in field order)

Every decoder returns (ok, fields) with ok False exactly where the Go
Unmarshal returns an error.  Field numbers are int32(key >> 3) as in Go.

Pinning: SCHEMAS (field numbers, wire types, embedded kinds) equals the
schema decoded from the reference's own FileDescriptorProto bytes
(raft.pb.go:698, descriptor_fields below; tests/golden/raftpb_schema.json),
which also exercises the decoder's nested-message path on reference bytes.
The encoder is cross-checked against Google's protobuf runtime (an
independent implementation of the same wire format, on a dynamically built
descriptor of raft.proto:68-86) in tests/test_wire_oracle.py, and the decoder
against the encoder and against hand-built malformed inputs for every error
path listed above.
"""
from __future__ import annotations

M64 = (1 << 64) - 1


class WireError(Exception):
    pass


def _varint(b: bytes, i: int, l: int):
    """The generated decoders' inline varint loop: shift up to 63, error at
    shift >= 64 (ErrIntOverflowRaft) or end of slice (io.ErrUnexpectedEOF)."""
    v = 0
    shift = 0
    while True:
        if shift >= 64:
            raise WireError("overflow")
        if i >= l:
            raise WireError("eof")
        c = b[i]
        i += 1
        v |= ((c & 0x7F) << shift) & M64
        if c < 0x80:
            return v, i
        shift += 7


def _as_int64(v: int) -> int:
    """Go's `int` (64-bit two's complement) of a varint accumulated in int."""
    return v - (1 << 64) if v >= (1 << 63) else v


def _int32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def skip_raft(b: bytes, i: int, l: int) -> int:
    """raft.pb.go:2909-2988 on dAtA[i:l]; returns the new index."""
    start = i
    depth = 0
    while i < l:
        wire, i = _varint(b, i, l)
        wt = wire & 7
        if wt == 0:
            shift = 0
            while True:
                if shift >= 64:
                    raise WireError("overflow")
                if i >= l:
                    raise WireError("eof")
                i += 1
                if b[i - 1] < 0x80:
                    break
                shift += 7
        elif wt == 1:
            i += 8
        elif wt == 2:
            length, i = _varint(b, i, l)
            length = _as_int64(length)
            if length < 0:
                raise WireError("invalid length")
            i += length
        elif wt == 3:
            depth += 1
        elif wt == 4:
            if depth == 0:
                raise WireError("unexpected end of group")
            depth -= 1
        elif wt == 5:
            i += 4
        else:
            raise WireError("illegal wiretype")
        if i - start < 0:
            raise WireError("invalid length")
        if depth == 0:
            return i
    raise WireError("eof")


def _len_field(b, i, l):
    n, i = _varint(b, i, l)
    n = _as_int64(n)
    if n < 0:
        raise WireError("invalid length")
    post = i + n
    if post > l:
        raise WireError("eof")
    return i, post


# schema: field -> ("v" varint | "b" bytes | ("m", kind) nested | "r" repeated
# uint64 (packed or not))
SCHEMAS = {
    "Message": {1: "v", 2: "v", 3: "v", 4: "v", 5: "v", 6: "v", 7: ("m", "Entry"), 8: "v",
                9: ("m", "Snapshot"), 10: "v", 11: "v", 12: "b"},
    "Entry": {1: "v", 2: "v", 3: "v", 4: "b"},
    "Snapshot": {1: "b", 2: ("m", "SnapshotMetadata")},
    "SnapshotMetadata": {1: ("m", "ConfState"), 2: "v", 3: "v"},
    "ConfState": {1: "r", 2: "r", 3: "r", 4: "r", 5: "v"},
}


def unmarshal(kind: str, b: bytes, i: int = 0, l: int = None, schemas: dict = None) -> dict:
    """Generic restatement of the generated Unmarshal methods above on
    dAtA[i:l]; raises WireError where Go returns an error.  Returns the last
    value of every varint field, bytes fields, and counts of nested/repeated
    elements.  ``schemas`` (default SCHEMAS) names the message kinds."""
    if l is None:
        l = len(b)
    if schemas is None:
        schemas = SCHEMAS
    schema = schemas[kind]
    out = {}
    while i < l:
        pre = i
        wire, i = _varint(b, i, l)
        fnum = _int32(wire >> 3)
        wt = wire & 7
        if wt == 4:
            raise WireError("end group for non-group")
        if fnum <= 0:
            raise WireError("illegal tag")
        kind_f = schema.get(fnum)
        if kind_f is None:
            i = pre
            i = skip_raft(b, i, l)
            if i > l:
                raise WireError("eof")
            continue
        if kind_f == "v":
            if wt != 0:
                raise WireError("wrong wiretype")
            v, i = _varint(b, i, l)
            out[fnum] = v
        elif kind_f == "b":
            if wt != 2:
                raise WireError("wrong wiretype")
            s, post = _len_field(b, i, l)
            out[fnum] = bytes(b[s:post])
            i = post
        elif kind_f == "r":
            vals = out.setdefault(fnum, [])
            if wt == 0:
                v, i = _varint(b, i, l)
                vals.append(v)
            elif wt == 2:
                s, post = _len_field(b, i, l)
                i = s
                while i < post:
                    v, i = _varint(b, i, l)  # bounded by l, not post (as written)
                    vals.append(v)
            else:
                raise WireError("wrong wiretype")
        else:
            if wt != 2:
                raise WireError("wrong wiretype")
            s, post = _len_field(b, i, l)
            sub = unmarshal(kind_f[1], b, s, post, schemas)
            out.setdefault(fnum, []).append(sub)
            i = post
    return out


# --------------------------------------------- the reference's descriptor ---
# raft.pb.go:698 holds raft.proto's FileDescriptorProto (gzipped), the one
# protobuf blob of raftpb the reference ships.  Decoding it with the decoder
# above (google/protobuf/descriptor.proto's schema, restated for the fields
# read here, plus gogoproto's (nullable) field option, gogo.proto: 65001)
# yields the field numbers, wire types and non-nullable embedded messages of
# the reference's own schema, against which SCHEMAS is pinned
# (tests/golden/make_raftpb_schema.py, tests/test_wire_oracle.py).
DESCRIPTOR_SCHEMAS = {
    "FileDescriptorProto": {1: "b", 2: "b", 4: ("m", "DescriptorProto")},
    "DescriptorProto": {1: "b", 2: ("m", "FieldDescriptorProto"),
                        3: ("m", "DescriptorProto")},
    "FieldDescriptorProto": {1: "b", 3: "v", 4: "v", 5: "v", 6: "b",
                             8: ("m", "FieldOptions")},
    "FieldOptions": {2: "v", 65001: "v"},
}
# FieldDescriptorProto.Type (descriptor.proto) -> wire type
_TYPE_WIRE = {1: 1, 2: 5, 3: 0, 4: 0, 5: 0, 6: 1, 7: 5, 8: 0, 9: 2, 11: 2, 12: 2, 13: 0, 14: 0,
              15: 5, 16: 1, 17: 0, 18: 0}
LABEL_REPEATED = 3
TYPE_MESSAGE = 11


def descriptor_fields(fdp: bytes) -> dict:
    """{message: {field number: {"name", "type", "label", "wire", "type_name",
    "nullable"}}} of a FileDescriptorProto, decoded with unmarshal()."""
    f = unmarshal("FileDescriptorProto", fdp, schemas=DESCRIPTOR_SCHEMAS)
    out = {}
    for m in f.get(4, []):
        fields = {}
        for fd in m.get(2, []):
            opts = (fd.get(8) or [{}])[-1]
            fields[int(fd[3])] = {
                "name": fd[1].decode(), "type": int(fd[5]), "label": int(fd[4]),
                "wire": _TYPE_WIRE[int(fd[5])], "type_name": fd.get(6, b"").decode(),
                "nullable": bool(opts.get(65001, 1)), "packed": bool(opts.get(2, 0))}
        out[m[1].decode()] = fields
    return out


def schema_from_descriptor(fields: dict, kinds=("Message", "Entry", "Snapshot",
                                                "SnapshotMetadata", "ConfState")) -> dict:
    """The SCHEMAS form of descriptor_fields() for the given messages:
    "v" varint scalar, "b" bytes, "r" repeated varint, ("m", kind) embedded
    message (a repeated or non-nullable embedded message decodes the same)."""
    out = {}
    for k in kinds:
        sch = {}
        for num, fd in fields[k].items():
            if fd["type"] == TYPE_MESSAGE:
                sch[num] = ("m", fd["type_name"].rsplit(".", 1)[-1])
            elif fd["label"] == LABEL_REPEATED and fd["wire"] == 0:
                sch[num] = "r"
            elif fd["wire"] == 0:
                sch[num] = "v"
            elif fd["wire"] == 2:
                sch[num] = "b"
            else:
                raise ValueError(f"{k}.{fd['name']}: wire type {fd['wire']} not in SCHEMAS' forms")
        out[k] = sch
    return out


def decode_message(b: bytes):
    """(ok, fields) — Message.Unmarshal."""
    try:
        return True, unmarshal("Message", b)
    except WireError:
        return False, None


# ------------------------------------------------------------- encoder ---

def varint(v: int) -> bytes:
    v &= M64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _key(f, wt):
    return varint((f << 3) | wt)


def marshal_conf_state(voters=(), learners=(), voters_outgoing=(), learners_next=(),
                       auto_leave=False) -> bytes:
    """ConfState.MarshalToSizedBuffer (raft.pb.go): repeated fields unpacked,
    auto_leave always written."""
    out = b""
    for f, vals in ((1, voters), (2, learners), (3, voters_outgoing), (4, learners_next)):
        for v in vals:
            out += _key(f, 0) + varint(v)
    out += _key(5, 0) + varint(1 if auto_leave else 0)
    return out


def marshal_snapshot(data=None, index=0, term=0, conf_state=b"") -> bytes:
    meta = _key(1, 2) + varint(len(conf_state)) + conf_state + _key(2, 0) + varint(index) + \
        _key(3, 0) + varint(term)
    out = b""
    if data is not None:
        out += _key(1, 2) + varint(len(data)) + data
    return out + _key(2, 2) + varint(len(meta)) + meta


def marshal_entry(term=0, index=0, etype=0, data=None) -> bytes:
    out = _key(1, 0) + varint(etype) + _key(2, 0) + varint(term) + _key(3, 0) + varint(index)
    if data is not None:
        out += _key(4, 2) + varint(len(data)) + data
    return out


EMPTY_SNAPSHOT = marshal_snapshot(conf_state=marshal_conf_state())


def marshal_message(type=0, to=0, frm=0, term=0, log_term=0, index=0, entries=(), commit=0,
                    snapshot=EMPTY_SNAPSHOT, reject=False, reject_hint=0, context=None) -> bytes:
    """Message.MarshalToSizedBuffer (raft.pb.go:903-972): every non-nullable
    field is written, in field-number order; Context only when non-nil."""
    out = _key(1, 0) + varint(type) + _key(2, 0) + varint(to) + _key(3, 0) + varint(frm) + \
        _key(4, 0) + varint(term) + _key(5, 0) + varint(log_term) + _key(6, 0) + varint(index)
    for e in entries:
        out += _key(7, 2) + varint(len(e)) + e
    out += _key(8, 0) + varint(commit)
    out += _key(9, 2) + varint(len(snapshot)) + snapshot
    out += _key(10, 0) + varint(1 if reject else 0)
    out += _key(11, 0) + varint(reject_hint)
    if context is not None:
        out += _key(12, 2) + varint(len(context)) + context
    return out


# --------------------------------------------------- ingest (the path) ---

KIND_OF_TYPE = {4: 0, 9: 1, 11: 2, 10: 3}  # MsgAppResp, MsgHeartbeatResp, MsgSnapStatus, MsgUnreachable
ST_OK, ST_UNMARSHAL, ST_TYPE, ST_CTX = 0, 1, 2, 3
NO_PROGRESS = 0x40


def ingest(b: bytes, group: int, ids):
    """One raw message -> (status, group, flags, index, term, hint, log_term,
    msg_type) as the wire-ingest kernel defines it: From is
    mapped to its slot among the group's sorted voter/learner ``ids`` (a
    non-member keeps NO_PROGRESS, as stepLeader drops it, raft.go:1099-1104);
    MsgHeartbeatResp's Context must be empty or 8 bytes (big-endian request
    id, non-zero)."""
    ok, f = decode_message(b)
    if not ok:
        return (ST_UNMARSHAL, 0xFFFFFFFF, 0, 0, 0, 0, 0, 0)
    mtype = _int32(f.get(1, 0))
    if mtype not in KIND_OF_TYPE:
        return (ST_TYPE, 0xFFFFFFFF, 0, 0, 0, 0, 0, mtype & 0xFF)
    kind = KIND_OF_TYPE[mtype]
    frm = f.get(3, 0)
    slot = NO_PROGRESS
    for s, vid in enumerate(ids):
        if vid == frm:
            slot = s
            break
    flags = (slot if slot != NO_PROGRESS else NO_PROGRESS) | (kind << 4) | (0x80 if f.get(10, 0) else 0)
    index = f.get(6, 0)
    if kind == 1:
        ctx = f.get(12, b"")
        if len(ctx) == 0:
            index = 0
        elif len(ctx) == 8 and int.from_bytes(ctx, "big") != 0:
            index = int.from_bytes(ctx, "big")
        else:
            return (ST_CTX, 0xFFFFFFFF, 0, 0, 0, 0, 0, mtype)
    return (ST_OK, group, flags, index, f.get(4, 0), f.get(11, 0), f.get(5, 0), mtype)
