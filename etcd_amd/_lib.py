"""ctypes binding of libquorumbatch.so (the C ABI in include/quorum_batch.h).

The library is built in-tree (``make -C etcd_amd/csrc`` or
``__graft_entry__.build()``).  There is no fallback: if the shared object is
missing every product entry point raises ``QuorumBatchError`` — the batch
engine never silently computes on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# The product library is always the in-tree build.  An A/B lab run selects
# another build explicitly (use_lab_library, from a `--lab-lib PATH` flag of
# bench.py / tools/bench_configs.py); no environment variable swaps it.
LIB_PATH = os.path.join(_HERE, "libquorumbatch.so")
_lab_path = None
_skipped: set = set()

QB_OK = 0
QB_EINVAL = -1
QB_EHIP = -2
QB_ENOMEM = -3

QB_MAX_SLOTS = 16
QB_WIDE_MAX_SLOTS = 1024
QB_REC_REJECT = 0x80
QB_STAT_NAMES = ("applied", "rejected", "stale_term", "non_member", "higher_term",
                 "bad_group", "after_stepdown")
QB_STAT_COUNT = 8
QB_VSTAT_NAMES = ("recorded", "duplicate", "stale_term", "higher_term", "after_stepdown", "bad",
                  "after_decision")
QB_VOTE_MODE_VOTE = 0
QB_VOTE_MODE_PREVOTE = 1


class QuorumBatchError(RuntimeError):
    pass


_u64, _u32, _i32, _p, _u64p = C.c_uint64, C.c_uint32, C.c_int, C.c_void_p, C.c_void_p

# name -> (restype, argtypes); must list exactly the functions the header declares.
SIGNATURES = {
    "qb_abi_version": (_i32, []),
    "qb_last_error": (C.c_char_p, []),
    "qb_device_count": (_i32, []),
    "qb_set_device": (_i32, [_i32]),
    "qb_malloc": (_i32, [C.c_size_t, C.POINTER(C.c_void_p)]),
    "qb_free": (_i32, [_p]),
    "qb_memset_async": (_i32, [_p, _i32, C.c_size_t, _p]),
    "qb_copy_h2d_async": (_i32, [_p, _p, C.c_size_t, _p]),
    "qb_copy_d2h_async": (_i32, [_p, _p, C.c_size_t, _p]),
    "qb_stream_create": (_i32, [C.POINTER(C.c_void_p)]),
    "qb_stream_destroy": (_i32, [_p]),
    "qb_stream_sync": (_i32, [_p]),
    "qb_host_compile_configs": (_i32, [_u64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _u64, _p]),
    "qb_dev_fixed_committed_vote": (_i32, [_u32, _u64, _p, _p, _p, _p, _p, _p]),
    "qb_dev_fixed_committed_vote_batches": (_i32, [_u32, _u64, _u32, _p, _p, _u32]),
    "qb_dev_csr_committed_vote": (_i32, [_u64, _u32, _p, _p, _p, _p, _p, _p, _p]),
    "qb_dev_csr_validate": (_i32, [_u64, _u32, _p, _p, _p]),
    "qb_dev_csr_committed_vote_checked": (_i32, [_u64, _u32, _p, _p, _p, _p, _p, _p, _p, _p]),
    "qb_dev_wide_committed_vote": (_i32, [_u64, _u32, _p, _p, _p, _p, _p, _p]),
    "qb_dev_wide_validate": (_i32, [_u64, _u32, _p, _p, _p]),
    "qb_dev_csr_quorum_active": (_i32, [_u64, _p, _p, _p, _p]),
    "qb_dev_fixed_apply_appresp": (_i32, [_u32, _u64, _u64, _p, _p, _p, _p, _p, _p, _p, _p,
                                          _p, _p, _p]),
    "qb_dev_fixed_commit_advance": (_i32, [_u32, _u64, _p, _p, _p, _p, _p]),
    "qb_dev_stepdown_check_armed": (_i32, [_u64, _p, _p, _p]),
    "qb_fixed_tracker_workspace_bytes": (C.c_size_t, [_u32, _u64, _u64]),
    "qb_dev_fixed_tracker_step": (_i32, [_u32, _u64, _u64] + [_p] * 14 + [C.c_size_t, _p]),
    "qb_dev_fixed_tracker_bucket": (_i32, [_u32, _u64, _u64] + [_p] * 5 + [C.c_size_t, _p]),
    "qb_dev_fixed_tracker_apply": (_i32, [_u32, _u64, _u64] + [_p] * 14 + [C.c_size_t, _p]),
    "qb_csr_tracker_workspace_bytes": (C.c_size_t, [_u64, _u32, _u64]),
    "qb_dev_csr_tracker_step": (_i32, [_u64, _u32, _p, _p, _u64] + [_p] * 14 + [C.c_size_t, _p]),
    "qb_votes_workspace_bytes": (C.c_size_t, [_u64]),
    "qb_dev_record_votes": (_i32, [_i32, _u64, _u64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                   C.c_size_t, _p]),
    "qb_dev_csr_tally_votes": (_i32, [_u64, _p, _p, _p, _p, _p, _p]),
    "qb_leader_workspace_bytes": (C.c_size_t, [_u64, _u64]),
    "qb_dev_leader_step": (_i32, [_p, _p, _p, _u64, _p, _p, _p, _p, _p, _p, C.c_size_t, _p]),
    "qb_leader_outbox_workspace_bytes": (C.c_size_t, [_u64, _u64]),
    "qb_dev_leader_step_outbox": (_i32, [_p, _p, _p, _p, _p, _p, _p, C.c_size_t, _p]),
    "qb_dev_ingest_messages": (_i32, [_u64, _p, _u64, _p, _p, _u64, _p, _p, _p, _p, _p, _p, _p,
                                      _p, _p, _p, _p, _p]),
    "qb_wire_group_rows_bytes": (C.c_size_t, [_u64]),
    "qb_dev_wire_group_rows": (_i32, [_u64, _p, _p, _p, _p]),
    "qb_dev_ingest_messages_rows": (_i32, [_u64, _p, _u64, _p, _p, _u64, _p, _p, _p, _p, _p,
                                           _p, _p, _p, _p, _p, _p, _p]),
    "qb_wire_fixed_tracker_workspace_bytes": (C.c_size_t, [_u32, _u64, _u64]),
    "qb_dev_ingest_fixed_tracker_step": (_i32, [_u32, _u64, _u64, _p, _u64] + [_p] * 17 +
                                         [C.c_size_t, _p]),
    "qb_wire_csr_tracker_workspace_bytes": (C.c_size_t, [_u64, _u32, _u64]),
    "qb_dev_ingest_csr_tracker_step": (_i32, [_u64, _u32, _p, _p, _u64, _p, _u64] + [_p] * 16 +
                                       [C.c_size_t, _p]),
    "qb_conf_change_workspace_bytes": (C.c_size_t, [_u64]),
    "qb_dev_conf_change": (_i32, [_p, _p, _p, C.c_size_t, _p]),
    "qb_shard_range": (_i32, [_u64, _i32, _i32, _p, _p]),
    "qb_comm_get_unique_id": (_i32, [_p]),
    "qb_comm_init": (_i32, [C.POINTER(C.c_void_p), _i32, _i32, _p]),
    "qb_comm_destroy": (_i32, [_p]),
    "qb_allgather_workspace_bytes": (C.c_size_t, [_u64, _i32]),
    "qb_dev_allgather_results": (_i32, [_p, _u64, _p, _p, _p, _p, _p, C.c_size_t, _p]),
    "qb_compact_changed_workspace_bytes": (C.c_size_t, [_u64]),
    "qb_dev_compact_changed": (_i32, [_u64, _p, _p, _u64, _p, _p, _p, _p, C.c_size_t, _p]),
    "qb_dev_scatter_changed": (_i32, [_u64, _p, _p, _u64, _p, _p]),
    "qb_allgather_changed_workspace_bytes": (C.c_size_t, [_u64, _i32]),
    "qb_dev_allgather_changed": (_i32, [_p, _u64, _p, _p, _p, _p, _p, C.c_size_t, _p]),
    "qb_route_partition_workspace_bytes": (C.c_size_t, [_i32, _u64]),
    "qb_dev_route_partition": (_i32, [_u64, _i32, _u64] + [_p] * 14 + [C.c_size_t, _p]),
    "qb_route_workspace_bytes": (C.c_size_t, [_i32, _u64]),
    "qb_dev_route_records": (_i32, [_p, _u64, _u64] + [_p] * 12 + [_u64, _p, _p, C.c_size_t, _p]),
    "qb_dev_synth_fixed": (_i32, [_u64, _u32, _u64, _u64, _p, _p, _p, _p, _p]),
    "qb_host_synth_csr_offsets": (_i32, [_u64, _u64, _u64, _p]),
    "qb_host_synth_joint_offsets": (_i32, [_u64, _u64, _u64, _p]),
    "qb_dev_synth_csr": (_i32, [_u64, _i32, _u64, _u64, _p, _p, _p, _p, _p]),
}

_lib = None
_lock = threading.Lock()


def use_lab_library(path: str) -> None:
    """Test/lab hook: bind ``path`` (an A/B build of the same ABI) instead of
    the in-tree library.  Must run before the first ``load()``.  Symbols the
    lab build lacks are recorded; ``call`` raises naming them."""
    global _lab_path
    if _lib is not None:
        raise QuorumBatchError("use_lab_library() after the library was loaded")
    if not os.path.exists(path):
        raise QuorumBatchError(f"lab library {path} does not exist")
    _lab_path = os.path.abspath(path)


def load() -> C.CDLL:
    """Load (once) and type the library; raises QuorumBatchError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _lab_path or LIB_PATH
        if not os.path.exists(path):
            raise QuorumBatchError(
                f"{path} not built: run `make -C etcd_amd/csrc` (or "
                "__graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if _lab_path and not hasattr(lib, name):  # an A/B build may predate newer symbols
                _skipped.add(name)
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.qb_abi_version() != 1:
            raise QuorumBatchError("libquorumbatch ABI version mismatch")
        if _skipped:
            import warnings
            warnings.warn(f"lab library {path} lacks {len(_skipped)} ABI symbol(s): "
                          f"{', '.join(sorted(_skipped))}", stacklevel=2)
        _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != QB_OK:
        msg = load().qb_last_error().decode(errors="replace")
        raise QuorumBatchError(f"{what} failed (rc={rc}): {msg}")


def fn(name: str):
    """The typed entry point ``name``; a symbol a lab build lacks raises here
    (never an untyped ctypes default that would truncate 64-bit pointers)."""
    lib = load()
    if name in _skipped:
        raise QuorumBatchError(f"{name} is missing from the lab library {_lab_path}")
    if name not in SIGNATURES:
        raise QuorumBatchError(f"{name} is not part of the ABI (include/quorum_batch.h)")
    return getattr(lib, name)


def call(name: str, *args) -> None:
    check(fn(name)(*args), name)
