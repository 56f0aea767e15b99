"""The C ABI library loads, exports exactly what include/quorum_batch.h
declares, and its host-side entry points behave without a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from etcd_amd import _lib
from etcd_amd.quorum import batch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "quorum_batch.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qb_\w+)\s*\(", text)))


def test_header_declares_what_binding_types():
    assert header_functions() == sorted(_lib.SIGNATURES)


def header_arity():
    """name -> number of parameters of each declaration in the header."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(qb_\w+)\s*\(([^;{)]*)\)\s*;", text):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_binding_arity_matches_header():
    """Every ctypes binding takes exactly the header's parameter count (an
    argument past the argtypes would be passed as a C int: a truncated
    stream or pointer)."""
    ar = header_arity()
    assert sorted(ar) == header_functions()
    bad = {k: (ar[k], len(v[1])) for k, v in _lib.SIGNATURES.items() if ar[k] != len(v[1])}
    assert not bad, bad


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name


def test_exported_symbols_in_dynsym():
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    exported = set(re.findall(r"\bT (qb_\w+)", out))
    assert set(header_functions()) <= exported


def test_version_and_devices():
    lib = _lib.load()
    assert lib.qb_abi_version() == 1
    assert lib.qb_device_count() >= 0


def test_errors_are_reported_not_raised():
    lib = _lib.load()
    rc = lib.qb_dev_fixed_committed_vote(17, 10, None, None, None, None, None, None)
    assert rc == _lib.QB_EINVAL
    assert b"0..16" in lib.qb_last_error()
    with pytest.raises(_lib.QuorumBatchError):
        _lib.call("qb_dev_fixed_apply_appresp", 0, 1, 1, *([None] * 10), None)
    # nothing to do is not an error, even without a device
    assert lib.qb_dev_fixed_committed_vote(5, 0, None, None, None, None, None, None) == 0


def test_host_offset_overflow_is_einval():
    lib = _lib.load()
    off = np.empty(2, np.uint32)
    assert lib.qb_host_synth_csr_offsets(1, 1, 0, off.ctypes.data) == 0
    assert 3 <= off[1] <= 11
    assert lib.qb_host_synth_csr_offsets(1, 1, 0, None) == _lib.QB_EINVAL


def test_compile_configs_slots_and_masks():
    cc = batch.compile_configs([{3, 1, 2}, {5}, set()], [{2, 4}, set(), set()],
                               [{7}, {6, 9}, set()])
    assert cc.off.tolist() == [0, 5, 8, 8]
    assert cc.slots(0).tolist() == [1, 2, 3, 4, 7]
    assert cc.cfg[0] == (0b00111 | (0b01010 << 16))
    assert cc.slots(1).tolist() == [5, 6, 9]
    assert cc.cfg[1] == 0b001
    assert cc.cfg[2] == 0 and cc.slots(2).size == 0


def test_compile_rejects_learner_voter_overlap():
    with pytest.raises(ValueError):
        batch.compile_configs([{1, 2}], [set()], [{2}])
    with pytest.raises(ValueError):
        batch.compile_configs([set(range(17))])


def test_product_refuses_cpu_tensors():
    import torch
    with pytest.raises(_lib.QuorumBatchError):
        batch.FixedGroups(5, 4, device="cpu")


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.QuorumBatchError, match="no CPU fallback"):
        _lib.load()


def _py_compile(vi, vo, lr):
    """tracker.Config -> slots/masks restated in Python (tracker.go:27-78,
    majority.go:106-113)."""
    slot = sorted(set(vi) | set(vo) | set(lr))
    m_in = sum(1 << j for j, i in enumerate(slot) if i in set(vi))
    m_out = sum(1 << j for j, i in enumerate(slot) if i in set(vo))
    return slot, m_in | (m_out << 16)


def test_host_compile_configs_random_vs_python():
    """qb_host_compile_configs (the C ABI config compile a cgo embedder calls)
    equals the Python restatement on random joint configs with learners and
    duplicate IDs, across the multi-thread threshold (65536 groups)."""
    rng = np.random.default_rng(11)
    G = 70000
    vi, vo, lr = [], [], []
    for g in range(G):
        ids = rng.choice(np.arange(1, 40), size=12, replace=False).tolist()
        a = int(rng.integers(0, 6))
        b = int(rng.integers(0, 6)) if rng.random() < 0.3 else 0
        c = int(rng.integers(0, 3))
        inc = ids[:a] + ids[:a][:1]              # a duplicate ID in the list
        out = ids[max(0, a - 2):max(0, a - 2) + b]
        vi.append(inc)
        vo.append(out)
        lr.append(ids[8:8 + c])
    cc = batch.compile_configs(vi, vo, lr)
    for g in rng.integers(0, G, size=3000).tolist() + [0, G - 1]:
        slot, cfg = _py_compile(vi[g], vo[g], lr[g])
        assert cc.slots(g).tolist() == slot and int(cc.cfg[g]) == cfg


def test_host_compile_configs_errors_name_the_reference_invariant():
    with pytest.raises(ValueError, match=r"group 1: 3 is in Learners and Voters\[0\]"):
        batch.compile_configs([{1}, {2, 3}], [set(), set()], [set(), {3, 9}])
    with pytest.raises(ValueError, match=r"group 0: 4 is in Learners and Voters\[1\]"):
        batch.compile_configs([{1, 4}], [{4, 5}], [{4}])
    with pytest.raises(ValueError, match=r"more than 16 members"):
        batch.compile_configs([set(range(1, 10))], [set(range(10, 18))])
    lib = _lib.load()
    off = np.array([0, 1], np.uint32)
    ids = np.array([7], np.uint64)
    o = np.zeros(2, np.uint32)
    c = np.zeros(1, np.uint32)
    out = np.zeros(1, np.uint64)
    # slot_cap too small is an error, a sizing call (slot_ids NULL) is not
    assert lib.qb_host_compile_configs(1, off.ctypes.data, ids.ctypes.data, None, None, None,
                                       None, o.ctypes.data, c.ctypes.data, None, 0, None) == 0
    assert o.tolist() == [0, 1] and c.tolist() == [1]
    assert lib.qb_host_compile_configs(1, off.ctypes.data, ids.ctypes.data, None, None, None,
                                       None, o.ctypes.data, c.ctypes.data, out.ctypes.data, 0,
                                       None) == _lib.QB_EINVAL


def test_shard_range_matches_python():
    """qb_shard_range (C ABI) == etcd_amd.shard.shard_range for every rank."""
    from etcd_amd.shard import shard_range
    lib = _lib.load()
    b, e = C.c_uint64(), C.c_uint64()
    for total, world in ((0, 1), (7, 3), (1 << 27, 8), (1000003, 8), (5, 8)):
        for r in range(world):
            assert lib.qb_shard_range(total, world, r, C.byref(b), C.byref(e)) == 0
            assert (b.value, e.value) == shard_range(total, world, r)
    assert lib.qb_shard_range(10, 2, 2, C.byref(b), C.byref(e)) == _lib.QB_EINVAL


def test_fake_rccl_library_covers_every_rccl_import():
    """tests/fake_rccl/libqb_fakecomm.so (test-only, the -m gpu
    test_gpu_comm_fake.py multi-rank tests) defines every nccl* symbol the
    product library imports from librccl, exports the same qb_* ABI, and
    does not itself depend on librccl."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prod = os.path.join(root, "etcd_amd", "libquorumbatch.so")
    fake = os.path.join(root, "tests", "fake_rccl", "libqb_fakecomm.so")

    def syms(path, kind):
        out = subprocess.run(["nm", "-D", path], capture_output=True, text=True, check=True).stdout
        return {ln.split()[-1] for ln in out.splitlines() if ln.split()[-2:-1] == [kind]}
    need = {s for s in syms(prod, "U") if s.startswith("nccl")}
    assert need, "the product library should import RCCL entry points"
    have = syms(fake, "T")
    assert need <= have, need - have
    assert {s for s in syms(prod, "T") if s.startswith("qb_")} <= have
    ldd = subprocess.run(["ldd", fake], capture_output=True, text=True).stdout
    assert "rccl" not in ldd


def test_tracker_region_grid_u32_guard():
    """The bucketed tracker steps address their reserved regions (about 2 x M
    records) with u32 offsets: a batch past that has no workspace size (0)
    and the step refuses it with QB_EINVAL before touching the device
    (G = 2^30 with M = 2^31 would wrap the region offsets)."""
    lib = _lib.load()
    assert lib.qb_fixed_tracker_workspace_bytes(5, 1 << 24, 1 << 24) > 0
    assert lib.qb_fixed_tracker_workspace_bytes(5, 1 << 30, 1 << 31) == 0
    assert lib.qb_csr_tracker_workspace_bytes(1 << 24, 8, 1 << 24) > 0
    assert lib.qb_csr_tracker_workspace_bytes(1 << 30, 8, 1 << 31) == 0
    dummy = C.c_void_p(0x1000)  # never dereferenced: the check fails first
    rc = lib.qb_dev_fixed_tracker_step(5, 1 << 30, 1 << 31, dummy, dummy, dummy, dummy, dummy,
                                       dummy, dummy, None, dummy, dummy, dummy, None, dummy,
                                       dummy, C.c_size_t(1 << 62), None)
    assert rc == _lib.QB_EINVAL
    assert b"region records" in lib.qb_last_error()
    rc = lib.qb_dev_csr_tracker_step(1 << 30, 8, dummy, dummy, 1 << 31, dummy, dummy, dummy, dummy,
                                     dummy, dummy, dummy, None, dummy, dummy, dummy, None, dummy,
                                     dummy, C.c_size_t(1 << 62), None)
    assert rc == _lib.QB_EINVAL
    assert b"region records" in lib.qb_last_error()


def test_composed_tick_validates_before_the_device():
    """qb_dev_ingest_{fixed,csr}_tracker_step refuse malformed arguments with
    QB_EINVAL and the reason before any HIP call (no GPU needed): slot counts
    out of range, a misaligned row table, no slot IDs at all, a batch past
    the u32 region grid, a short workspace; their workspace sizes are the
    tracker step's plus the two escape columns, 0 where no workspace fits."""
    lib = _lib.load()
    M = 1 << 24
    assert (lib.qb_wire_fixed_tracker_workspace_bytes(5, M, M)
            >= lib.qb_fixed_tracker_workspace_bytes(5, M, M) + 16 * M)
    assert lib.qb_wire_fixed_tracker_workspace_bytes(0, 16, 16) == 0
    assert lib.qb_wire_fixed_tracker_workspace_bytes(17, 16, 16) == 0
    assert lib.qb_wire_fixed_tracker_workspace_bytes(5, 1 << 30, 1 << 31) == 0
    assert (lib.qb_wire_csr_tracker_workspace_bytes(M, 8, M)
            >= lib.qb_csr_tracker_workspace_bytes(M, 8, M) + 16 * M)
    assert lib.qb_wire_csr_tracker_workspace_bytes(16, 17, 16) == 0
    d = C.c_void_p(0x1000)  # never dereferenced: each check fails first

    def fixed(n, G, M_, rows=d, off=None, ids=None, ws_bytes=1 << 40):
        return lib.qb_dev_ingest_fixed_tracker_step(
            n, G, M_, d, 100, d, d, rows, off, ids, d, d, d, None, d, d, d, None, d, None, d, d,
            C.c_size_t(ws_bytes), None)
    cases = [(lambda: fixed(0, 16, 16), b"n must be"),
             (lambda: fixed(5, 16, 16, rows=C.c_void_p(0x1008)), b"16-byte aligned"),
             (lambda: fixed(5, 16, 16, rows=None), b"rows, or off and ids"),
             (lambda: fixed(5, 1 << 30, 1 << 31), b"region records"),
             (lambda: fixed(5, 16, 16, ws_bytes=8), b"workspace too small")]
    for call, why in cases:
        rc = call()
        assert rc == _lib.QB_EINVAL, why
        assert why in lib.qb_last_error(), (why, lib.qb_last_error())
    rc = lib.qb_dev_ingest_csr_tracker_step(16, 8, d, d, 16, d, 100, d, d, None, None, d, d, d,
                                            None, d, d, d, None, d, None, d, d, C.c_size_t(1 << 40),
                                            None)
    assert rc == _lib.QB_EINVAL and b"required" in lib.qb_last_error()
    rc = lib.qb_dev_ingest_csr_tracker_step(16, 17, d, d, 16, d, 100, d, d, None, d, d, d, d,
                                            None, d, d, d, None, d, None, d, d, C.c_size_t(1 << 40),
                                            None)
    assert rc == _lib.QB_EINVAL and b"max_slots" in lib.qb_last_error()


def test_leader_outbox_binding_layout_matches_header(tmp_path):
    """The Python binding's qb_leader_outbox / qb_read_state match the
    header's layout (gcc on the header itself): the ReadState area's two
    fields sit where the library reads them."""
    import subprocess
    from etcd_amd.quorum.leader import READ_STATE_DTYPE, LeaderOutboxC
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "quorum_batch.h"\n'
                   'int main(void) { printf("%zu %zu %zu %zu\\n", sizeof(qb_leader_outbox), '
                   'offsetof(qb_leader_outbox, read_states), offsetof(qb_leader_outbox, read_count), '
                   'sizeof(qb_read_state)); return 0; }\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert got == [C.sizeof(LeaderOutboxC), LeaderOutboxC.read_states.offset,
                   LeaderOutboxC.read_count.offset, READ_STATE_DTYPE.itemsize]


def test_leader_state_arrays_checked_before_any_device_work():
    """LeaderGroups refuses a state table with a missing or short array (the
    C ABI would read past it on the device) before it touches a device."""
    import numpy as np
    from etcd_amd.quorum import leader
    G, n, K = 4, 3, 4
    arrays = {k: np.zeros(1, dt) for k, dt in leader.GROUP_ARRAYS.items()}
    arrays["off"] = np.arange(0, n * G + 1, n, dtype=np.uint32)
    arrays["cfg"] = np.zeros(G, np.uint32)
    for k in ("meta", "term", "committed", "first_index", "last_index", "snap_index",
              "snap_term", "max_ents"):
        arrays[k] = np.zeros(G, leader.GROUP_ARRAYS[k])
    for k in ("run_start", "run_term"):
        arrays[k] = np.zeros(G * leader.MAX_RUNS, np.uint64)
    for k in ("match", "next", "pending_snapshot", "pstate", "infl_pos"):
        arrays[k] = np.zeros(n * G, leader.GROUP_ARRAYS[k])
    arrays["infl_buf"] = np.zeros(n * G * K, np.uint64)
    # complete: only the device is refused
    with pytest.raises(_lib.QuorumBatchError, match="HIP device"):
        leader.LeaderGroups(arrays, K, device="cpu")
    short = dict(arrays, infl_buf=np.zeros(n * G * K - 1, np.uint64))
    with pytest.raises(_lib.QuorumBatchError, match="infl_buf"):
        leader.LeaderGroups(short, K, device="cpu")
    with pytest.raises(_lib.QuorumBatchError, match="rq_ctx"):
        leader.LeaderGroups(arrays, K, readq_cap=2, device="cpu")
    ring = dict(arrays, infl_pos=np.full(n * G, K << 16, np.uint32))  # full rings: valid
    with pytest.raises(_lib.QuorumBatchError, match="HIP device"):
        leader.LeaderGroups(ring, K, device="cpu")
    for bad in (K, (K + 1) << 16):  # start past the ring, count past it
        ring["infl_pos"] = np.zeros(n * G, np.uint32)
        ring["infl_pos"][7] = bad
        with pytest.raises(_lib.QuorumBatchError, match=r"infl_pos\[7\]"):
            leader.LeaderGroups(ring, K, device="cpu")
    with pytest.raises(_lib.QuorumBatchError, match="inflight_cap"):
        leader.LeaderGroups(arrays, 0, device="cpu")
    missing = {k: v for k, v in arrays.items() if k != "match"}
    with pytest.raises(_lib.QuorumBatchError, match="match"):
        leader.LeaderGroups(missing, K, device="cpu")


def test_tensor_checks_refuse_host_tensors_and_bad_counts():
    import torch
    from etcd_amd.quorum import _checks, leader
    with pytest.raises(_lib.QuorumBatchError, match="device tensor"):
        _checks.check_tensors(((torch.zeros(4, dtype=torch.int64), "x", _checks.I64, 4),))
    _checks.check_tensors(((None, "omitted", _checks.I64, 4),))
    z = torch.zeros(1)
    ib = leader.LeaderInbox(z, z, z, z, z, z)
    ib._m = -1
    with pytest.raises(_lib.QuorumBatchError, match="non-negative"):
        ib.check()
