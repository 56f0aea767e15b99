"""Step-by-step probe of etcd_amd.comm.RcclComm on a single-rank group
(development tool): prints a line after every call, so a hang names its
step.  Usage: python tools/lab/rccl_world1.py {nccl|gloo} [side]
("side": the calls run on a created stream instead of the null stream)."""
import faulthandler
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
faulthandler.dump_traceback_later(60, exit=True)
backend = sys.argv[1] if len(sys.argv) > 1 else "nccl"
side = len(sys.argv) > 2 and sys.argv[2] == "side"
t0 = time.time()


def say(what):
    print(f"{time.time() - t0:7.2f}s {what}", flush=True)


os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"))
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
if backend == "nccl":
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
else:
    dist.init_process_group("gloo", rank=0, world_size=1)
say(f"init_process_group({backend})")
if side:
    torch.cuda.set_stream(torch.cuda.Stream(dev))
say(f"current stream {torch.cuda.current_stream(dev).cuda_stream:#x}")
from etcd_amd.comm import RcclComm  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402
uid = RcclComm.unique_id()
say("qb_comm_get_unique_id")
box = [uid]
dist.broadcast_object_list(box, src=0)
say("broadcast_object_list")
comm = RcclComm(1, 0, dev, box[0])
say("qb_comm_init")
grp = batch.FixedGroups.synth(3, 5, 50_000, device=dev)
c, v = grp.committed_vote()
gc, gv = comm.allgather_results(c, v, 50_000)
torch.cuda.synchronize()
say(f"qb_dev_allgather_results ok={bool(torch.equal(gc, c)) and bool(torch.equal(gv, v))}")
M = 10_000
cols = {"group": torch.randint(0, 50_005, (M,), device=dev),
        "flags": torch.randint(0, 5, (M,), device=dev).to(torch.uint8),
        "index": torch.arange(M, device=dev, dtype=torch.int64),
        "term": torch.full((M,), 7, dtype=torch.int64, device=dev)}
got = comm.route_records(cols, 50_000)
torch.cuda.synchronize()
say(f"qb_dev_route_records count={got['group'].numel()}")
comm.close()
say("qb_comm_destroy")
dist.destroy_process_group()
say("done")
