"""Random raftpb message generator for the wire-ingest tests (valid, minimal,
unknown-field, truncated and mutated encodings).  Test infrastructure."""
import numpy as np

from oracle import raftpb_ref as W


def rand_u64(r):
    return r.choice([0, 1, 5, 127, 128, 300, 1 << 32, (1 << 63) - 1, 1 << 63, (1 << 64) - 1,
                     r.getrandbits(64), r.getrandbits(30)])


def random_message(r, ids):
    t = r.choice([4, 4, 4, 9, 9, 10, 11, 3, 6, 18])
    frm = r.choice(ids) if ids and r.random() < 0.9 else rand_u64(r)
    ctx = None
    if t == 9 and r.random() < 0.7:
        ctx = r.choice([b"", r.getrandbits(64).to_bytes(8, "big"), b"\x00" * 8, b"abc"])
    ents = [W.marshal_entry(rand_u64(r), rand_u64(r), r.randint(0, 2),
                            bytes(r.getrandbits(8) for _ in range(r.randint(0, 4))))
            for _ in range(r.choice([0, 0, 0, 1, 2]))]
    snap = W.EMPTY_SNAPSHOT
    if r.random() < 0.1:
        snap = W.marshal_snapshot(b"xy", rand_u64(r), rand_u64(r),
                                  W.marshal_conf_state([1, 2, 3], [4], [5], [], True))
    b = W.marshal_message(t, rand_u64(r), frm, rand_u64(r), rand_u64(r), rand_u64(r), ents,
                          rand_u64(r), snap, r.random() < 0.4, rand_u64(r), ctx)
    x = r.random()
    if x < 0.05:  # unknown fields before/after
        b = W._key(77, 0) + W.varint(9) + b + W._key(78, 2) + b"\x01z"
    elif x < 0.10:  # truncation
        b = b[: r.randint(0, len(b))]
    elif x < 0.18:  # random byte mutation
        bb = bytearray(b)
        for _ in range(r.randint(1, 3)):
            if bb:
                bb[r.randrange(len(bb))] = r.getrandbits(8)
        b = bytes(bb)
    elif x < 0.20:  # minimal encodings (google-style: only set fields)
        b = W._key(1, 0) + W.varint(t) + W._key(3, 0) + W.varint(frm) + W._key(6, 0) + W.varint(7)
    elif x < 0.26:  # fields repeated after the canonical run (the last one wins)
        extra = r.choice([(1, r.choice([4, 9, 11, 3])), (3, frm), (4, rand_u64(r)), (6, rand_u64(r)),
                          (10, r.randint(0, 1)), (11, rand_u64(r))])
        b = b + W._key(extra[0], 0) + W.varint(extra[1])
    elif x < 0.30:  # canonical run broken midway (a field moved to the front)
        b = W._key(6, 0) + W.varint(rand_u64(r)) + b
    return b


def groups_ids(r, G):
    off = [0]
    ids = []
    for _ in range(G):
        k = r.randint(1, 16)
        s = sorted(r.sample(range(1, 10_000), k))
        ids += s
        off.append(off[-1] + k)
    return np.array(off, np.uint32), np.array(ids, np.uint64)


