"""Wire ingest (include/quorum_batch.h ``qb_dev_ingest_messages``): raw
protobuf raftpb.Message bytes (raft/raftpb/raft.proto:68-86) decoded on the
device into leader-inbox records for ``LeaderGroups.step``.  Validation is
the generated gogoproto Message.Unmarshal (raftpb/raft.pb.go:1739-2061)."""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib
from .leader import LeaderInbox

WIRE_OK, WIRE_UNMARSHAL, WIRE_TYPE, WIRE_CTX = 0, 1, 2, 3
REC_NO_PROGRESS = 0x40


def pack_messages(msgs, groups, device="cuda"):
    """Host helper: a list of encoded messages and their envelope groups ->
    (bytes u8, msg_off int64 [M+1], msg_group int32) device tensors."""
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs), np.uint8) if msgs else np.zeros(0, np.uint8)
    dev = torch.device(device)
    b = torch.from_numpy(buf.copy() if buf.size else np.zeros(1, np.uint8)).to(dev)
    return (b, int(off[-1]), torch.from_numpy(off.view(np.int64).copy()).to(dev),
            torch.from_numpy(np.asarray(groups, np.uint32).view(np.int32).copy()).to(dev))


def ingest(buf: torch.Tensor, nbytes: int, msg_off: torch.Tensor, msg_group: torch.Tensor,
           off: torch.Tensor, ids: torch.Tensor, stats: torch.Tensor = None):
    """Decode M = len(msg_group) messages.  ``off`` [G+1] int32 and ``ids``
    [off[G]] int64 are the groups' CSR slot IDs (ascending per group).
    Returns (LeaderInbox, status u8 tensor, msg_type u8 tensor)."""
    for t, what in ((buf, "buf"), (msg_off, "msg_off"), (msg_group, "msg_group")):
        if not t.is_cuda:
            raise _lib.QuorumBatchError(f"{what} must be a device tensor; there is no CPU path")
    dev = buf.device
    M = msg_group.numel()
    G = off.numel() - 1
    n = max(M, 1)
    rg = torch.empty(n, dtype=torch.int32, device=dev)
    rf = torch.empty(n, dtype=torch.uint8, device=dev)
    ri, rt, rh, rl = (torch.empty(n, dtype=torch.int64, device=dev) for _ in range(4))
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    mtype = torch.empty(n, dtype=torch.uint8, device=dev)
    _lib.call("qb_dev_ingest_messages", M, buf.data_ptr(), nbytes, msg_off.data_ptr(),
              msg_group.data_ptr(), G, off.data_ptr(), ids.data_ptr(), rg.data_ptr(),
              rf.data_ptr(), ri.data_ptr(), rt.data_ptr(), rh.data_ptr(), rl.data_ptr(),
              status.data_ptr(), mtype.data_ptr(), None if stats is None else stats.data_ptr(),
              torch.cuda.current_stream(dev).cuda_stream)
    ib = LeaderInbox(rg, rf, ri, rt, rh, rl)
    ib._m = M
    return ib, status[:M], mtype[:M]
