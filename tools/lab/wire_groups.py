"""Lab: wire ingest time vs the number of groups (random off/ids lookups
from L2 vs from HBM/MALL).  Development only."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from etcd_amd.quorum import wire  # noqa: E402

dev = torch.device("cuda")
M = 1 << 24
for G in (1 << 12, 1 << 18, M // 4):
    buf, moff, grp, off, ids = wire.synth_response_stream(M, G)
    d = [torch.from_numpy(x).to(dev) for x in (buf, moff.view(np.int64), grp.view(np.int32),
                                                 off.view(np.int32), ids.view(np.int64))]
    nb = int(moff[-1])
    for _ in range(3):
        wire.ingest(d[0], nb, d[1], d[2], d[3], d[4])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        wire.ingest(d[0], nb, d[1], d[2], d[3], d[4])
    e1.record()
    torch.cuda.synchronize()
    print(f"G={G:9d} per call {e0.elapsed_time(e1) / 10 * 1000:8.1f} us", flush=True)
