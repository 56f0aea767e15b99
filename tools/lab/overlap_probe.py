"""Lab probe (GPU, development only): does the wire decode of tick k+1 overlap
with the tracker apply of tick k on one MI355X?  Times, on the composed
workload (tools/bench_configs.py wire_tracker_tick, 16M groups):
  ingest   wire.ingest (k_ingest + deferred) alone
  step     the tracker step on the decoded records alone
  both     the two on two streams at once (independent data)
and prints per-call microseconds.  If `both` is near max(ingest, step) a
split composed call (decode+bucket | apply) pipelined over ticks would pay;
near the sum it would not."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench_configs as bc  # noqa: E402
from etcd_amd.quorum import batch, wire  # noqa: E402


def main():
    dev = torch.device("cuda")
    G = 1 << 24
    tr, snap, ticks, rows, off, ids = bc.wire_tracker_tick(G, 2, dev_=dev)
    buf, nbytes, moff, grp, direct = ticks[1]
    ib, _, _ = wire.ingest(*ticks[0][:4], off, ids, rows=rows)
    rec = batch.AppRespBatch(ib.group, ib.flags, ib.index, ib.term)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def restore():
        for k, v in snap.items():
            getattr(tr, k).copy_(v)

    def t_ingest():
        wire.ingest(buf, nbytes, moff, grp, off, ids, rows=rows)

    def t_step():
        tr.step(rec, reset_stats=False, rearm=False)

    def t_both():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            t_ingest()
        t_step()
        main_s.wait_stream(side)

    out = {}
    for name, fn in (("ingest", t_ingest), ("step", t_step), ("both", t_both),
                     ("ingest", t_ingest), ("step", t_step), ("both", t_both)):
        best = float("inf")
        for _ in range(5):
            restore()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 10 * 1e6)
        out[name] = min(out.get(name, best), best)
        print(name, round(best, 1), "us", flush=True)
    print(json.dumps({k: round(v, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
