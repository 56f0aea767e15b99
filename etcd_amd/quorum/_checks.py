"""Argument checks of the Python mirror before a C-ABI call.  The ABI takes
plain device pointers (include/quorum_batch.h), so a short, strided or
mistyped tensor handed through would be read or written past its end on the
device; every wrapper checks its tensors here first and raises
QuorumBatchError instead."""
from __future__ import annotations

import torch

from .. import _lib


def check_tensors(specs) -> None:
    """specs: (tensor, name, dtypes, min elements) each — a contiguous device
    tensor of one of ``dtypes`` with at least that many elements (a None
    tensor is an omitted optional argument and is skipped); all on one
    device."""
    dev = None
    for t, what, dts, n_min in specs:
        if t is None:
            continue
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise _lib.QuorumBatchError(f"{what} must be a device tensor; there is no CPU path")
        if t.dtype not in dts or not t.is_contiguous() or t.numel() < n_min:
            raise _lib.QuorumBatchError(
                f"{what} must be a contiguous {'/'.join(str(d) for d in dts)} device tensor of "
                f">= {n_min} elements (got {t.dtype}, {t.numel()} elements"
                f"{'' if t.is_contiguous() else ', strided'})")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise _lib.QuorumBatchError(f"{what} is on {t.device}, the call's other tensors on {dev}")


I64 = (torch.int64,)
I32 = (torch.int32,)
I16 = (torch.int16,)
U8 = (torch.uint8,)
FLAG = (torch.uint8, torch.bool)
