#!/usr/bin/env python3
"""Generate tests/golden/raftpb_schema.json from the reference's own bytes.

The reference ships raft.proto's FileDescriptorProto, gzipped, as a byte
literal in raft/raftpb/raft.pb.go (`fileDescriptor_b042552c306ae59b`,
raft.pb.go:698).  This script reads that literal, gunzips it and decodes it
with the oracle's restated wire decoder (oracle/raftpb_ref.py
descriptor_fields), cross-checks every field against Google's protobuf
runtime parsing the same bytes (descriptor_pb2), and writes the decoded
schema of Message, Entry, Snapshot, SnapshotMetadata and ConfState — field
numbers, names, types, labels, wire types, gogoproto (nullable) — as the
fixture.  The blob itself is not stored.

    python tests/golden/make_raftpb_schema.py [/root/reference]
"""
import gzip
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import raftpb_ref as r  # noqa: E402

KINDS = ("Message", "Entry", "Snapshot", "SnapshotMetadata", "ConfState")
VAR = "fileDescriptor_b042552c306ae59b"


def reference_descriptor(ref_root: str) -> bytes:
    src = open(os.path.join(ref_root, "raft", "raftpb", "raft.pb.go")).read()
    i = src.index(f"var {VAR} = []byte{{")
    body = src[src.index("{", i) + 1:src.index("}", i)]
    return gzip.decompress(bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", body)))


def decoded_schema(fdp: bytes) -> dict:
    f = r.descriptor_fields(fdp)
    return {k: {str(n): f[k][n] for n in sorted(f[k])} for k in KINDS}


def cross_check(fdp: bytes, schema: dict) -> None:
    """Google's runtime parses the same bytes to the same fields."""
    from google.protobuf import descriptor_pb2
    fd = descriptor_pb2.FileDescriptorProto()
    fd.ParseFromString(fdp)
    byname = {m.name: m for m in fd.message_type}
    for k in KINDS:
        got = {str(x.number): (x.name, x.type, x.label, x.type_name) for x in byname[k].field}
        want = {n: (v["name"], v["type"], v["label"], v["type_name"]) for n, v in schema[k].items()}
        assert got == want, (k, got, want)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    fdp = reference_descriptor(ref)
    schema = decoded_schema(fdp)
    cross_check(fdp, schema)
    out = {"source": f"raft/raftpb/raft.pb.go:698 ({VAR}, gzipped FileDescriptorProto, "
                     f"{len(fdp)} bytes decoded)", "messages": schema}
    path = os.path.join(ROOT, "tests", "golden", "raftpb_schema.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
