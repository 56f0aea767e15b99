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
