"""Lab probe driver (development tool): times tools/lab/k5_ceiling.hip's
variants over 16M groups with HIP events; prints one line per variant."""
import ctypes as C
import os
import sys

import torch

G = 1 << 24
lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bin", "libk5_ceiling.so"))
dev = torch.device("cuda", 0)
rec = torch.randint(0, 1 << 62, (G,), device=dev)
chain = torch.randperm(G // 512, device=dev).to(torch.int32)
gterm = torch.full((G,), 7, dtype=torch.int64, device=dev)
ts = torch.randint(0, 1 << 40, (G,), device=dev)
match = torch.randint(0, 1 << 40, (5, G), device=dev)
committed = torch.zeros(G, dtype=torch.int64, device=dev)
active = torch.zeros(G, dtype=torch.int16, device=dev)
st = torch.cuda.current_stream().cuda_stream
names = {0: "stream", 1: "+lds apply", 2: "+apply+chain1", 3: "+apply+chain2",
         4: "+chain2 no apply", 5: "loads only"}
rb, wb = 74, 42   # bytes per group read / written
for rnd in range(3):
    for v in names:
        args = (v, C.c_uint64(G), C.c_void_p(rec.data_ptr()), C.c_void_p(chain.data_ptr()),
                C.c_void_p(gterm.data_ptr()), C.c_void_p(ts.data_ptr()), C.c_void_p(match.data_ptr()),
                C.c_void_p(committed.data_ptr()), C.c_void_p(active.data_ptr()), C.c_void_p(st))
        for _ in range(5):
            assert lib.lab_k5_ceiling(*args) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 50
        e0.record()
        for _ in range(K):
            lib.lab_k5_ceiling(*args)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / K
        by = G * (rb + (wb if v != 5 else 0))
        print(f"{names[v]:18s} {us:8.1f} us  {by / us / 1e6:6.2f} TB/s  ({by / 1e9:.2f} GB)", flush=True)
sys.exit(0)
