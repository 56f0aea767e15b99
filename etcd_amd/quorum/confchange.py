"""Batched configuration changes (include/quorum_batch.h
``qb_dev_conf_change``): one confchange.Changer operation per group —
Simple / EnterJoint / LeaveJoint over its ConfChangeSingle list
(raft/confchange/confchange.go:49-334) — for G groups in one call, producing
the new CSR config and carried / initialised Progress.  Restore(ConfState)
(raft/confchange/restore.go:116-155) is ``restore`` below: the same calls in
the reference's order."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from .. import _lib

NONE, SIMPLE, ENTER_JOINT, ENTER_JOINT_AUTOLEAVE, LEAVE_JOINT = 0, 1, 2, 3, 4
ADD_NODE, REMOVE_NODE, UPDATE_NODE, ADD_LEARNER = 0, 1, 2, 3

ERR_MESSAGES = {
    1: "config is already joint", 2: "can't make a zero-voter config joint",
    3: "can't leave a non-joint config", 4: "can't apply simple config change in joint config",
    5: "more than one voter changed without entering joint config", 6: "removed all voters",
    7: "unexpected conf type {}", 8: "no progress for {}",
    9: "{} is in LearnersNext, but not Voters[1]",
    10: "{} is in LearnersNext, but is already marked as learner",
    11: "{} is in Learners and Voters[1]", 12: "{} is in Learners and Voters[0]",
    13: "{} is in Learners, but is not marked as learner",
    14: "AutoLeave must be false when not joint", 15: "more than 16 members, or 24 alive within one change (engine limit)",
    16: "bad operation",
}

_P = C.c_void_p
SLOT_ARRAYS = {"ids": np.uint64, "match": np.uint64, "next": np.uint64,
               "pending_snapshot": np.uint64, "pstate": np.uint8, "infl_pos": np.uint32}
_SIGNED = {np.uint8: np.uint8, np.uint32: np.int32, np.uint64: np.int64}


class _In(C.Structure):
    _fields_ = [("G", C.c_uint64), ("inflight_cap", C.c_uint32), ("reserved", C.c_uint32)] + [
        (n, _P) for n in ("op", "cc_off", "cc_type", "cc_node", "last_index", "off", "ids", "cfg",
                          "ext", "match", "next", "pending_snapshot", "pstate", "infl_pos",
                          "infl_buf")]


class _Out(C.Structure):
    _fields_ = [("slot_cap", C.c_uint64)] + [
        (n, _P) for n in ("new_off", "ids", "cfg", "ext", "match", "next", "pending_snapshot",
                          "pstate", "infl_pos", "infl_buf", "err", "err_id")]


def error_text(code: int, err_id: int) -> str:
    msg = ERR_MESSAGES.get(code, f"error {code}")
    return msg.format(err_id) if "{}" in msg else msg


def _dev(a, dt, device):
    a = np.ascontiguousarray(np.asarray(a, dtype=dt))
    if a.size == 0:
        a = np.zeros(1, dt)
    return torch.from_numpy(a.view(_SIGNED[dt]).copy()).to(device)


# ``out`` of change_soa: element size per key; per-slot arrays share the slot
# capacity, infl_buf holds capacity x K, the per-group ones G (new_off G + 1).
_OUT_ELEM = {"new_off": 4, "cfg": 4, "ext": 4, "err": 1, "err_id": 8, "ids": 8, "match": 8,
             "next": 8, "pending_snapshot": 8, "pstate": 1, "infl_pos": 4, "infl_buf": 8}
_OUT_SLOT = ("ids", "match", "next", "pending_snapshot", "pstate", "infl_pos")


def _check_out(o: Dict[str, torch.Tensor], G: int, K: int, dev, table) -> int:
    """Validate caller-owned outputs before their raw pointers reach
    qb_dev_conf_change: the kernels write slot_cap entries of
    every per-slot array, slot_cap x K of infl_buf and G (+1) of the per-group
    ones, so a short, strided, host, wrongly sized or aliased tensor would be
    an out-of-bounds or self-overwriting device write.  Returns slot_cap =
    the shortest per-slot array."""
    missing = [k for k in _OUT_ELEM if k not in o]
    if missing:
        raise _lib.QuorumBatchError(f"conf change out: missing {missing}")
    for k, es in _OUT_ELEM.items():
        t = o[k]
        if not isinstance(t, torch.Tensor) or t.device != dev:
            raise _lib.QuorumBatchError(f"conf change out[{k!r}]: a tensor on {dev} is required")
        if t.element_size() != es:
            raise _lib.QuorumBatchError(
                f"conf change out[{k!r}]: element size {t.element_size()}, expected {es}")
        if not t.is_contiguous():
            raise _lib.QuorumBatchError(f"conf change out[{k!r}]: must be contiguous")
    cap = min(o[k].numel() for k in _OUT_SLOT)
    if cap < 1:
        raise _lib.QuorumBatchError("conf change out: per-slot arrays are empty")
    if o["infl_buf"].numel() < max(1, cap * K):
        raise _lib.QuorumBatchError(
            f"conf change out['infl_buf']: {o['infl_buf'].numel()} < slot capacity {cap} x {K}")
    for k, n in (("new_off", G + 1), ("cfg", G), ("ext", G), ("err", G), ("err_id", G)):
        if o[k].numel() < n:
            raise _lib.QuorumBatchError(f"conf change out[{k!r}]: {o[k].numel()} < {n}")

    def span(t):
        a = t.data_ptr()
        return a, a + t.numel() * t.element_size()
    outs = [(k, span(o[k])) for k in _OUT_ELEM]
    ins = [(k, span(v)) for k, v in table.items()]
    for i, (ka, (a0, a1)) in enumerate(outs):
        for kb, (b0, b1) in outs[i + 1:] + ins:
            if a0 < b1 and b0 < a1:
                raise _lib.QuorumBatchError(f"conf change out[{ka!r}] overlaps {kb!r}")
    return cap


@dataclass
class ConfigTable:
    """G groups' configs (CSR slots) and Progress on one device."""
    G: int
    S: int
    inflight_cap: int
    t: Dict[str, torch.Tensor]

    @classmethod
    def from_numpy(cls, off, ids, cfg, ext, progress: Dict[str, np.ndarray], inflight_cap: int,
                   device="cuda"):
        dev = torch.device(device)
        if dev.type != "cuda":
            raise _lib.QuorumBatchError("ConfigTable needs a HIP device; there is no CPU path")
        G, S = len(cfg), int(off[-1])
        t = {"off": _dev(off, np.uint32, dev), "cfg": _dev(cfg, np.uint32, dev),
             "ext": _dev(ext, np.uint32, dev), "ids": _dev(ids, np.uint64, dev)}
        for k in ("match", "next", "pending_snapshot", "pstate", "infl_pos"):
            t[k] = _dev(progress[k], SLOT_ARRAYS[k], dev)
        t["infl_buf"] = _dev(progress.get("infl_buf", np.zeros(S * inflight_cap, np.uint64)),
                             np.uint64, dev)
        return cls(G, S, inflight_cap, t)

    def numpy(self) -> Dict[str, np.ndarray]:
        n = {"off": self.G + 1, "cfg": self.G, "ext": self.G, "infl_buf": self.S * self.inflight_cap}
        out = {}
        for k, v in self.t.items():
            dt = {"off": np.uint32, "cfg": np.uint32, "ext": np.uint32,
                  "infl_buf": np.uint64}.get(k, SLOT_ARRAYS.get(k))
            out[k] = v.cpu().numpy().view(dt)[: n.get(k, self.S)]
        return out

    def change(self, op: Sequence[int], ccs: Sequence[Sequence[Tuple[int, int]]],
               last_index: Sequence[int], out=None):
        """Apply op[g] with ccs[g] = [(ConfChangeType, NodeID), ...] to every
        group; returns (new ConfigTable, err u8[G], err_id u64[G]).  ``out``:
        as ``change_soa``."""
        G = self.G
        cc_off = np.zeros(G + 1, np.uint32)
        cc_off[1:] = np.cumsum([len(c) for c in ccs])
        flat = [x for c in ccs for x in c]
        return self.change_soa(np.asarray(op, np.uint8), cc_off,
                               np.array([t for t, _ in flat], np.uint8),
                               np.array([n for _, n in flat], np.uint64),
                               np.asarray(last_index, np.uint64), out=out)

    def change_soa(self, op, cc_off, cc_type, cc_node, last_index, fetch_errors=True, out=None):
        """As ``change`` with the operation already in SoA form (numpy arrays
        or device tensors): op[G] u8, cc_off[G+1] u32, cc_type / cc_node per
        change, last_index[G] u64.  ``out`` (optional): caller-owned output
        tensors (the keys below; per-slot arrays of equal length = the slot
        capacity, infl_buf capacity x K)."""
        dev = self.t["off"].device
        G = self.G

        def d(a, dt):
            return a if isinstance(a, torch.Tensor) else _dev(a, dt, dev)
        d_op, d_ccoff = d(op, np.uint8), d(cc_off, np.uint32)
        d_cct, d_ccn, d_last = d(cc_type, np.uint8), d(cc_node, np.uint64), d(last_index, np.uint64)
        n_changes = int(d_ccoff[G].item()) if isinstance(cc_off, torch.Tensor) else int(cc_off[-1])
        cap = min(16 * G, self.S + n_changes) + 1
        K = self.inflight_cap
        o = {"new_off": torch.zeros(G + 1, dtype=torch.int32, device=dev),
             "ids": torch.empty(cap, dtype=torch.int64, device=dev),
             "cfg": torch.empty(G, dtype=torch.int32, device=dev),
             "ext": torch.empty(G, dtype=torch.int32, device=dev),
             "match": torch.empty(cap, dtype=torch.int64, device=dev),
             "next": torch.empty(cap, dtype=torch.int64, device=dev),
             "pending_snapshot": torch.empty(cap, dtype=torch.int64, device=dev),
             "pstate": torch.empty(cap, dtype=torch.uint8, device=dev),
             "infl_pos": torch.empty(cap, dtype=torch.int32, device=dev),
             "infl_buf": torch.empty(max(1, cap * K), dtype=torch.int64, device=dev),
             "err": torch.empty(G, dtype=torch.uint8, device=dev),
             "err_id": torch.empty(G, dtype=torch.int64, device=dev)}
        if out is not None:
            o = out
            cap = _check_out(o, G, K, dev, self.t)
        i = _In(G=G, inflight_cap=K, reserved=0)
        for k, v in (("op", d_op), ("cc_off", d_ccoff), ("cc_type", d_cct), ("cc_node", d_ccn),
                     ("last_index", d_last)):
            setattr(i, k, v.data_ptr())
        for k in ("off", "ids", "cfg", "ext", "match", "next", "pending_snapshot", "pstate",
                  "infl_pos", "infl_buf"):
            setattr(i, k, self.t[k].data_ptr())
        out = _Out(slot_cap=cap)
        for k, v in o.items():
            setattr(out, k, v.data_ptr())
        need = _lib.load().qb_conf_change_workspace_bytes(G)
        if getattr(self, "_ws", None) is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=dev)
        _lib.call("qb_dev_conf_change", C.byref(i), C.byref(out), self._ws.data_ptr(), need,
                  torch.cuda.current_stream(dev).cuda_stream)
        self._last_out = (i, out, o)  # keep the argument blocks alive until the stream is synced
        S_new = int(o["new_off"][G].item())
        if S_new > cap:
            raise _lib.QuorumBatchError(f"conf change needs {S_new} slots, capacity {cap}")
        t = {"off": o["new_off"], "cfg": o["cfg"], "ext": o["ext"]}
        for k in ("ids", "match", "next", "pending_snapshot", "pstate", "infl_pos", "infl_buf"):
            t[k] = o[k]
        nt = ConfigTable(G, S_new, K, t)
        if not fetch_errors:
            return nt, o["err"], o["err_id"]
        return (nt, o["err"].cpu().numpy(), o["err_id"].cpu().numpy().view(np.uint64))


def restore(table: ConfigTable, conf_states: List[dict], last_index: Sequence[int]):
    """confchange.Restore (restore.go:116-155) for every group at once:
    conf_states[g] = dict(voters, learners, voters_outgoing, learners_next,
    auto_leave).  Groups advance through the same call sequence (a group with
    fewer steps gets QB_CC_NONE); a group's first error stops it.  Returns
    (table, err, err_id)."""
    G = table.G
    plans = []
    for cs in conf_states:
        out = [(ADD_NODE, i) for i in cs.get("voters_outgoing", ())]
        inc = [(REMOVE_NODE, i) for i in cs.get("voters_outgoing", ())]
        inc += [(ADD_NODE, i) for i in cs.get("voters", ())]
        inc += [(ADD_LEARNER, i) for i in cs.get("learners", ())]
        inc += [(ADD_LEARNER, i) for i in cs.get("learners_next", ())]
        if not out:
            steps = [(SIMPLE, [cc]) for cc in inc]
        else:
            steps = [(SIMPLE, [cc]) for cc in out]
            steps.append((ENTER_JOINT_AUTOLEAVE if cs.get("auto_leave") else ENTER_JOINT, inc))
        plans.append(steps)
    err = np.zeros(G, np.uint8)
    err_id = np.zeros(G, np.uint64)
    for k in range(max((len(p) for p in plans), default=0)):
        op = [p[k][0] if k < len(p) and not err[g] else NONE for g, p in enumerate(plans)]
        ccs = [p[k][1] if k < len(p) and not err[g] else [] for g, p in enumerate(plans)]
        table, e, eid = table.change(op, ccs, last_index)
        fresh = (err == 0) & (e != 0)
        err[fresh], err_id[fresh] = e[fresh], eid[fresh]
    return table, err, err_id
