"""ctypes access to the C oracle (oracle/liborc_quorum.so) — tests/bench only.

Builds the library on first use if it is missing (gcc is on both the build
container and the GPU box).  Also provides numpy-level wrappers so tests can
compare the HIP engine with the oracle on identical seeded inputs.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_DIR = os.path.join(ROOT, "oracle")
ORC_PATH = os.path.join(ORC_DIR, "liborc_quorum.so")

_p, _u64, _u32, _i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
SIG = {
    "orc_gen_fixed": (None, [_u64, _u32, _u64, _u64, _p, _p, _p, _p]),
    "orc_gen_csr": (_i32, [_u64, _i32, _u64, _u64, _p, _p, _p, _p]),
    "orc_csr_eval": (None, [_u64, _p, _p, _p, _p, _p, _p]),
    "orc_fixed_eval": (None, [_u32, _u64, _p, _p, _p, _p, _p]),
    "orc_csr_quorum_active": (None, [_u64, _p, _p, _p]),
    "orc_wide_eval": (None, [_u64, _p, _p, _p, _p, _p]),
    "orc_group_maps_size": (C.c_size_t, []),
    "orc_faithful_build_fixed": (None, [_u32, _u64, _p, _p, _p, _p]),
    "orc_faithful_eval": (None, [_u64, _p, _p, _p]),
    "orc_faithful_eval_mt": (None, [_u64, _p, _p, _p, _i32]),
    "orc_joint_maps_size": (C.c_size_t, []),
    "orc_faithful_build_csr": (_i32, [_u64, _p, _p, _p, _p, _p]),
    "orc_faithful_joint_eval": (None, [_u64, _p, _p, _p]),
    "orc_faithful_joint_eval_mt": (None, [_u64, _p, _p, _p, _i32]),
    "orc_fixed_eval_mt": (None, [_u32, _u64, _p, _p, _p, _p, _p, _i32]),
    "orc_csr_eval_mt": (None, [_u64, _p, _p, _p, _p, _p, _p, _i32]),
    "orc_fixed_appresp_sequential": (_i32, [_u32, _u64, _u64, _p, _p, _p, _p, _p, _p, _p, _p,
                                            _p, _p, _p, _p, _p]),
    "orc_fixed_appresp_sequential_mt": (_i32, [_u32, _u64, _u64, _p, _p, _p, _p, _p, _p, _p,
                                               _p, _p, _p, _p, _p, _p, _i32]),
    "orc_csr_appresp_sequential": (_i32, [_u64, _p, _p, _u64, _p, _p, _p, _p, _p, _p, _p, _p,
                                          _p, _p, _p, _p, _p, _i32]),
    "orc_fixed_commit_all": (None, [_u32, _u64, _p, _p, _p, _p]),
    "orc_csr_commit_all": (None, [_u64, _p, _p, _p, _p, _p, _p]),
    "orc_bench_plumbing": (_u64, [_u32, _u64, _u64]),
    "orc_leader_step": (_u64, [_p, _p, _p, _u64, _p, _p, _p, _i32]),
    "orc_ingest": (None, [_u64, _p, _u64, _p, _p, _u64, _p, _p] + [_p] * 7 + [_i32]),
}

_lib = None


def load():
    global _lib
    if _lib is None:
        srcs = [os.path.join(ORC_DIR, f) for f in ("quorum_oracle.c", "leader_oracle.c", "wire_oracle.c")]
        if not os.path.exists(ORC_PATH) or any(os.path.getmtime(ORC_PATH) < os.path.getmtime(s)
                                                for s in srcs):
            subprocess.check_call(["make", "-s", "-C", ORC_DIR])
        lib = C.CDLL(ORC_PATH)
        for k, (r, a) in SIG.items():
            f = getattr(lib, k)
            f.restype = r
            f.argtypes = a
        _lib = lib
    return _lib


def ptr(a):
    return None if a is None else a.ctypes.data


def mask_np(n):
    return np.uint8 if n <= 8 else np.uint16


def gen_fixed(seed, n, G, g_begin=0):
    lib = load()
    match = np.empty((n, G), np.uint64)
    vd = np.empty(G, mask_np(n))
    gr = np.empty(G, mask_np(n))
    ts = np.empty(G, np.uint64)
    lib.orc_gen_fixed(seed, n, G, g_begin, ptr(match), ptr(vd), ptr(gr), ptr(ts))
    return match, vd, gr, ts


def gen_csr(seed, kind, G, g_begin=0):
    lib = load()
    off = np.empty(G + 1, np.uint32)
    # upper bound on slots: 11 (ragged) / 10 (joint)
    match = np.empty(G * 11 + 2, np.uint64)
    cfg = np.empty(G, np.uint32)
    votes = np.empty(G, np.uint32)
    rc = lib.orc_gen_csr(seed, {"ragged": 0, "joint": 1}[kind], G, g_begin, ptr(off), ptr(match),
                         ptr(cfg), ptr(votes))
    assert rc == 0
    return off, match[:off[-1]].copy(), cfg, votes


def fixed_eval(n, match, vd, gr, threads=1):
    lib = load()
    G = match.shape[1] if n else len(vd)
    commit = np.empty(G, np.uint64)
    vote = np.empty(G, np.uint8)
    if threads > 1:
        lib.orc_fixed_eval_mt(n, G, ptr(match), ptr(vd), ptr(gr), ptr(commit), ptr(vote), threads)
    else:
        lib.orc_fixed_eval(n, G, ptr(match), ptr(vd), ptr(gr), ptr(commit), ptr(vote))
    return commit, vote


def csr_eval(off, match, cfg, votes, threads=1):
    lib = load()
    G = len(cfg)
    commit = np.empty(G, np.uint64)
    vote = np.empty(G, np.uint8)
    m = match if match.size else np.zeros(1, np.uint64)
    if threads > 1:
        lib.orc_csr_eval_mt(G, ptr(off), ptr(m), ptr(cfg), ptr(votes), ptr(commit), ptr(vote),
                            threads)
    else:
        lib.orc_csr_eval(G, ptr(off), ptr(m), ptr(cfg), ptr(votes), ptr(commit), ptr(vote))
    return commit, vote


def wide_eval(off, match, flags):
    lib = load()
    G = len(off) - 1
    commit = np.empty(G, np.uint64)
    vote = np.empty(G, np.uint8)
    m = match if match.size else np.zeros(1, np.uint64)
    f = flags if flags.size else np.zeros(1, np.uint8)
    lib.orc_wide_eval(G, ptr(off), ptr(m), ptr(f), ptr(commit), ptr(vote))
    return commit, vote


def quorum_active(cfg, active):
    lib = load()
    won = np.empty(len(cfg), np.uint8)
    lib.orc_csr_quorum_active(len(cfg), ptr(cfg), ptr(active), ptr(won))
    return won


def faithful_maps(n, match, vd, gr):
    lib = load()
    G = match.shape[1]
    maps = np.empty(G * lib.orc_group_maps_size(), np.uint8)
    lib.orc_faithful_build_fixed(n, G, ptr(match), ptr(vd), ptr(gr), ptr(maps))
    return maps


def faithful_eval(maps, G, threads=1):
    lib = load()
    commit = np.empty(G, np.uint64)
    vote = np.empty(G, np.uint8)
    if threads > 1:
        lib.orc_faithful_eval_mt(G, ptr(maps), ptr(commit), ptr(vote), threads)
    else:
        lib.orc_faithful_eval(G, ptr(maps), ptr(commit), ptr(vote))
    return commit, vote


def faithful_csr_maps(off, match, cfg, votes):
    """Per-group Go-map tables of the CSR/joint form (oracle/quorum_oracle.c
    orc_faithful_build_csr): JointConfig maps, ProgressMap, votes map."""
    lib = load()
    G = len(cfg)
    maps = np.empty(max(G, 1) * lib.orc_joint_maps_size(), np.uint8)
    m = match if match.size else np.zeros(1, np.uint64)
    rc = lib.orc_faithful_build_csr(G, ptr(off), ptr(m), ptr(cfg), ptr(votes), ptr(maps))
    assert rc == 0, "a group has more than 11 slots"
    return maps


def faithful_joint_eval(maps, G, threads=1):
    lib = load()
    commit = np.empty(G, np.uint64)
    vote = np.empty(G, np.uint8)
    if threads > 1:
        lib.orc_faithful_joint_eval_mt(G, ptr(maps), ptr(commit), ptr(vote), threads)
    else:
        lib.orc_faithful_joint_eval(G, ptr(maps), ptr(commit), ptr(vote))
    return commit, vote


def appresp_sequential(n, G, rec, state, threads=1):
    """Sequential reference semantics; ``state`` (dict of numpy arrays) is
    updated in place.  Returns the stats array.  threads > 1 partitions the
    groups (each thread scans the batch for its own groups: the same result)."""
    lib = load()
    stats = np.zeros(8, np.uint64)
    group, flags, index, term = rec
    rc = lib.orc_fixed_appresp_sequential_mt(
        n, G, len(group), ptr(group), ptr(flags), ptr(index), ptr(term), ptr(state["term"]),
        ptr(state["term_start"]), ptr(state.get("last_index")), ptr(state["match"]),
        ptr(state.get("next")), ptr(state["active"]), ptr(state["committed"]),
        ptr(state["stepped_down"]), ptr(stats), threads)
    assert rc == 0, "a record acked past the leader's last index"
    return stats


def csr_appresp_sequential(off, cfg, rec, state, threads=1):
    """Sequential MsgAppResp semantics over the CSR layout (learners have a
    Progress, joint CommittedIndex); ``state`` updated in place."""
    lib = load()
    stats = np.zeros(8, np.uint64)
    group, flags, index, term = rec
    G = len(cfg)
    m = state["match"] if state["match"].size else np.zeros(1, np.uint64)
    nx = state.get("next")
    rc = lib.orc_csr_appresp_sequential(
        G, ptr(off), ptr(cfg), len(group), ptr(group), ptr(flags), ptr(index), ptr(term),
        ptr(state["term"]), ptr(state["term_start"]), ptr(state.get("last_index")), ptr(m),
        ptr(nx if nx is None or nx.size else np.zeros(1, np.uint64)), ptr(state["active"]),
        ptr(state["committed"]), ptr(state["stepped_down"]), ptr(stats), threads)
    assert rc == 0, "a record acked past the leader's last index"
    return stats


def csr_commit_all(off, cfg, match, term_start, committed):
    lib = load()
    G = len(committed)
    adv = np.empty(G, np.uint8)
    m = match if match.size else np.zeros(1, np.uint64)
    lib.orc_csr_commit_all(G, ptr(off), ptr(cfg), ptr(m), ptr(term_start), ptr(committed),
                           ptr(adv))
    return adv


def commit_all(n, match, term_start, committed):
    lib = load()
    G = len(committed)
    adv = np.empty(G, np.uint8)
    lib.orc_fixed_commit_all(n, G, ptr(match), ptr(term_start), ptr(committed), ptr(adv))
    return adv


# ----------------------------------------------------------- leader step ---

LEADER_FIELDS = ("off", "cfg", "meta", "term", "committed", "first_index", "last_index",
                 "snap_index", "snap_term", "max_ents", "run_start", "run_term", "match", "next",
                 "pending_snapshot", "pstate", "infl_pos", "infl_buf", "rq_ctx", "rq_index",
                 "rq_meta")


class _LG(C.Structure):
    _fields_ = [("G", C.c_uint64), ("K", C.c_uint32), ("Q", C.c_uint32),
                ("read_only", C.c_uint32), ("reserved", C.c_uint32)] + [(f, _p) for f in LEADER_FIELDS]


class _IN(C.Structure):
    _fields_ = [("M", C.c_uint64)] + [(f, _p) for f in ("group", "flags", "index", "term", "hint",
                                                         "log_term")]


LEADER_MSG_DTYPE = np.dtype([("index", "<u8"), ("log_term", "<u8"), ("commit", "<u8"),
                             ("aux", "<u8"), ("group", "<u4"), ("to", "u1"), ("type", "u1"),
                             ("reserved", "<u2")])


def leader_step(arrays, inflight_cap, readq_cap, read_only, rec, threads=1, msg_cap=None):
    """Sequential leader inbox step over SoA ``arrays`` (numpy, updated in
    place); ``rec`` = dict(group, flags, index, term, hint, log_term).
    Returns (msgs, total, stepdown_at, gflags, stats)."""
    lib = load()
    G = len(arrays["cfg"])
    keep = {k: np.ascontiguousarray(v) if v.size else np.zeros(1, v.dtype)
            for k, v in arrays.items()}
    for k in arrays:
        if arrays[k].size:
            assert keep[k] is arrays[k] or np.shares_memory(keep[k], arrays[k]), k
    lg = _LG(G=G, K=inflight_cap, Q=readq_cap, read_only=read_only, reserved=0)
    for f in LEADER_FIELDS:
        setattr(lg, f, keep[f].ctypes.data)
    M = len(rec["group"])
    z = np.zeros(1, np.uint64)
    ib = _IN(M=M)
    for f in ("group", "flags", "index", "term", "hint", "log_term"):
        a = rec.get(f)
        setattr(ib, f, (a if a is not None and a.size else z).ctypes.data)
    if msg_cap is None:
        msg_cap = 8 * M + 16
    msgs = np.zeros(msg_cap, LEADER_MSG_DTYPE)
    sd = np.empty(G, np.uint32)
    gf = np.empty(G, np.uint8)
    stats = np.zeros(8, np.uint64)
    total = lib.orc_leader_step(C.byref(lg), C.byref(ib), msgs.ctypes.data, msg_cap,
                                sd.ctypes.data, gf.ctypes.data, stats.ctypes.data, threads)
    return msgs[:min(total, msg_cap)], int(total), sd, gf, stats


def ingest(buf, moff, mgroup, off, ids, threads=1, nbytes=None):
    """Wire ingest restated (oracle/wire_oracle.c): returns dict of record
    columns + status.  nbytes: the buffer's length (default the last offset;
    given when the offsets are corrupt and may point past it)."""
    lib = load()
    M = len(mgroup)
    out = {"group": np.empty(M, np.uint32), "flags": np.empty(M, np.uint8),
           "index": np.empty(M, np.uint64), "term": np.empty(M, np.uint64),
           "hint": np.empty(M, np.uint64), "log_term": np.empty(M, np.uint64),
           "status": np.empty(M, np.uint8)}
    b = buf if buf.size else np.zeros(1, np.uint8)
    nb = int(moff[-1]) if nbytes is None else int(nbytes)
    assert nb <= buf.size or nb == 0, "nbytes past the host buffer"
    lib.orc_ingest(M, ptr(b), nb, ptr(moff), ptr(mgroup), len(off) - 1, ptr(off),
                   ptr(ids if ids.size else np.zeros(1, np.uint64)), ptr(out["group"]),
                   ptr(out["flags"]), ptr(out["index"]), ptr(out["term"]), ptr(out["hint"]),
                   ptr(out["log_term"]), ptr(out["status"]), threads)
    return out
