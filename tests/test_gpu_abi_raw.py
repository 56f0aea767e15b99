"""Drive the C ABI the way the Go cgo package does: its own
stream, device memory and copies — no torch — and compare with the oracle."""
import ctypes as C

import numpy as np
import pytest

from etcd_amd import _lib
from tests import oracle_c as oc

pytestmark = pytest.mark.gpu


class Dev:
    def __init__(self):
        self.lib = _lib.load()
        self.ptrs = []

    def alloc(self, nbytes):
        p = C.c_void_p()
        _lib.check(self.lib.qb_malloc(nbytes, C.byref(p)), "qb_malloc")
        self.ptrs.append(p.value)
        return p.value

    def close(self):
        for p in self.ptrs:
            _lib.check(self.lib.qb_free(p), "qb_free")


def test_fixed_roundtrip_raw_abi():
    lib = _lib.load()
    _lib.check(lib.qb_set_device(0), "qb_set_device")
    st = C.c_void_p()
    _lib.check(lib.qb_stream_create(C.byref(st)), "qb_stream_create")
    d = Dev()
    n, G = 5, 100003
    match, vd, gr, _ = oc.gen_fixed(0x5EED0002, n, G)
    dm, dvd, dgr = d.alloc(match.nbytes), d.alloc(G), d.alloc(G)
    dc, dv = d.alloc(8 * G), d.alloc(G)
    for dst, src in ((dm, match), (dvd, vd), (dgr, gr)):
        _lib.check(lib.qb_copy_h2d_async(dst, src.ctypes.data, src.nbytes, st), "h2d")
    _lib.check(lib.qb_memset_async(dc, 0, 8 * G, st), "memset")
    _lib.check(lib.qb_dev_fixed_committed_vote(n, G, dm, dvd, dgr, dc, dv, st), "eval")
    c = np.empty(G, np.uint64)
    v = np.empty(G, np.uint8)
    _lib.check(lib.qb_copy_d2h_async(c.ctypes.data, dc, c.nbytes, st), "d2h")
    _lib.check(lib.qb_copy_d2h_async(v.ctypes.data, dv, v.nbytes, st), "d2h")
    _lib.check(lib.qb_stream_sync(st), "sync")
    ec, ev = oc.fixed_eval(n, match, vd, gr)
    assert np.array_equal(c, ec) and np.array_equal(v, ev)
    d.close()
    _lib.check(lib.qb_stream_destroy(st), "qb_stream_destroy")


def test_malloc_reports_enomem():
    lib = _lib.load()
    p = C.c_void_p()
    rc = lib.qb_malloc(1 << 50, C.byref(p))  # 1 PiB
    assert rc in (_lib.QB_ENOMEM, _lib.QB_EHIP)
    assert lib.qb_last_error()
