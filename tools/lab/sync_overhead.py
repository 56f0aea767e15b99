"""Where the fixed wall-clock overhead of a short timed region goes (bench.py
with --steps 20): event records, the first launch, the final synchronise."""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import HipEvents  # noqa: E402
from etcd_amd import _lib  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402

FLAGS = int(os.environ.get("QB_LAB_DEVFLAGS", "-1"))
if FLAGS >= 0:  # before anything touches the device (hipDeviceScheduleSpin = 1, Yield = 2)
    _h = C.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags", FLAGS, "->", _h.hipSetDeviceFlags(C.c_uint(FLAGS)), flush=True)
dev = torch.device("cuda", 0)
lib = _lib.load()
G, n, B = 1 << 20, 5, 16
groups = [batch.FixedGroups.synth(0x5EED0002, n, G, g_begin=b * G, device=dev) for b in range(B)]
outs = [(torch.empty(G, dtype=torch.int64, device=dev), torch.empty(G, dtype=torch.uint8, device=dev))
        for _ in range(B)]
streams = [torch.cuda.Stream(dev) for _ in range(2)]
args = [[(n, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(), c.data_ptr(),
          v.data_ptr(), st.cuda_stream) for g, (c, v) in zip(groups, outs)] for st in streams]
fn = lib.qb_dev_fixed_committed_vote
hip = C.CDLL("libamdhip64.so")
hip.hipEventSynchronize.argtypes = [C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
for _ in range(20000):
    fn(*args[_ % 2][_ % B])
torch.cuda.synchronize()
ev = HipEvents(4)
K = 20
for mode in ("torch_sync", "event_sync", "event_torch"):
    rows = []
    for rep in range(30):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        for s_, st in enumerate(streams):
            ev.record(ev.ev[s_], st.cuda_stream)
        t.append(time.perf_counter())
        fn(*args[0][0])
        t.append(time.perf_counter())
        for k in range(1, K):
            fn(*args[k % 2][k % B])
        t.append(time.perf_counter())
        for s_, st in enumerate(streams):
            ev.record(ev.ev[2 + s_], st.cuda_stream)
        t.append(time.perf_counter())
        if mode == "torch_sync":
            torch.cuda.synchronize()
        elif mode == "device_sync":
            hip.hipDeviceSynchronize()
        elif mode == "event_sync":
            hip.hipEventSynchronize(ev.ev[2])
            hip.hipEventSynchronize(ev.ev[3])
        elif mode == "event_torch":
            hip.hipEventSynchronize(ev.ev[2])
            hip.hipEventSynchronize(ev.ev[3])
            torch.cuda.synchronize()
        else:
            for st in streams:
                hip.hipStreamSynchronize(st.cuda_stream)
        t.append(time.perf_counter())
        dev_us = max(ev.elapsed_ms(0, 2), ev.elapsed_ms(0, 3)) * 1e3 - min(0.0, ev.elapsed_ms(0, 1) * 1e3)
        rows.append([(t[i + 1] - t[i]) * 1e6 for i in range(5)] + [(t[-1] - t[0]) * 1e6, dev_us])
    rows.sort(key=lambda r: r[5])
    med = rows[len(rows) // 2]
    print(f"{mode:12s} rec0 {med[0]:6.1f} first {med[1]:6.1f} rest19 {med[2]:6.1f} rec1 {med[3]:6.1f} "
          f"sync {med[4]:6.1f} | wall {med[5]:6.1f} dev {med[6]:6.1f} us (K={K}) "
          f"wall/step {med[5]/K:5.2f} dev/step {med[6]/K:5.2f}", flush=True)
