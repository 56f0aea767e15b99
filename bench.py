#!/usr/bin/env python3
"""Benchmark: raft groups quorum-evaluated per second on MI355X.

Workload (BASELINE.json configs[1]): 1M (2^20) raft groups x 5 voters per GPU,
CommittedIndex + VoteResult fused in one kernel, uint64 match indexes, FIXED
slot-major SoA layout.  One step = one pass of the hot path over one batch
of 2^20 groups.  ``--batches`` distinct batches (default 16, ~0.96 GB with
outputs) stay resident in HBM and are visited round-robin, so every step
streams its batch from HBM instead of the 256 MB Infinity Cache (the
MALL-warm single-batch rate is reported beside it as ``value_mall_warm``).

Launch pipeline: consecutive steps are independent batches, so they are
issued round-robin on ``--streams`` HIP streams (default 2): the tail of one
launch overlaps the ramp of the next.  HIP events on the launch streams bracket
the timed region; the per-launch duration used for the roofline is the
region's device time / K.

``--workload ragged|joint`` runs BASELINE configs[2] / configs[3] instead
(16M ragged 3-9-voter groups with learners / 8M JointConfig 5+5 groups per
GPU, CSR layout, ``k_csr``) with the same timing and JSON contract; the default
stays configs[1], the metric's headline config.

Multi-GPU: one process per GPU (torch.distributed, RCCL), groups sharded by
global group number (weak scaling, no collective in the timed region); for
N > 1 the node-wide all-gather of one batch's commit/vote vectors is timed
separately (``allgather_ms``).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from etcd_amd import _lib  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402
from etcd_amd.shard import allgather_results  # noqa: E402

METRIC = "raft groups quorum-evaluated/sec (1 and 8 GPUs) + % peak HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0x5EED0002      # 0x5EED0001 + config#


def bytes_per_group(n: int) -> int:
    """Algorithmic bytes of the fused kernel per group:
    read match 8n + voted + granted masks, write commit 8 + vote 1."""
    mb = 1 if n <= 8 else 2
    return 8 * n + 2 * mb + 8 + 1


class HipEvents:
    """Raw hipEvent timing on an arbitrary stream (the stream the kernels are
    launched on); ~1 us of host time per record."""

    def __init__(self, count: int):
        self.hip = C.CDLL("libamdhip64.so")
        self.hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
        self.hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        self.hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        self.hip.hipEventDestroy.argtypes = [C.c_void_p]
        self.ev = []
        for _ in range(count):
            e = C.c_void_p()
            assert self.hip.hipEventCreate(C.byref(e)) == 0
            self.ev.append(e)
        self.record = self.hip.hipEventRecord

    def elapsed_ms(self, a: int, b: int) -> float:
        ms = C.c_float()
        assert self.hip.hipEventElapsedTime(C.byref(ms), self.ev[a], self.ev[b]) == 0
        return ms.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(e)


def load_traffic(workload_key: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (written by
    tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE passes of this
    same bench command, with the gfx950 FETCH_SIZE x2 correction)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(n: int, sample_groups: int, seconds: float):
    """The oracle's faithful C restatement of the Go loop (per-group hash-map
    MajorityConfig + AckedIndexer lookups + insertionSort, majority.go:126-210)
    timed on the host cores over a bounded sample of the same workload."""
    from tests import oracle_c as oc
    threads = max(1, min(16, os.cpu_count() or 1))
    match, vd, gr, _ = oc.gen_fixed(SEED, n, sample_groups)
    maps = oc.faithful_maps(n, match, vd, gr)

    def rate(th):
        reps, t0 = 0, time.perf_counter()
        while True:
            oc.faithful_eval(maps, sample_groups, threads=th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                return reps * sample_groups / dt, reps

    r1, reps1 = rate(1)
    rn, repsn = rate(threads)
    return {
        "value": rn, "unit": "groups/s", "cores": threads, "kind": "port",
        "sample": (f"{sample_groups} groups x {n} voters (same synthetic spec), faithful C "
                   f"restatement of majority.go CommittedIndex+VoteResult with Go-map-style "
                   f"hash lookups; {repsn} passes on {threads} threads (GOMAXPROCS-equivalent "
                   f"{threads}); 1 thread: {r1:.4g} groups/s over {reps1} passes"),
        "value_1thread": r1,
    }


def cpu_baseline_csr(kind: str, seconds: float):
    """The oracle's C SoA restatement (majority.go / joint.go per group) on a
    bounded 1M-group sample of the same CSR workload, 16 host threads."""
    from tests import oracle_c as oc
    threads = max(1, min(16, os.cpu_count() or 1))
    gs = 1 << 20
    seed = {"ragged": 0x5EED0003, "joint": 0x5EED0004}[kind]
    off, m, cfg, votes = oc.gen_csr(seed, kind, gs)
    reps, t0 = 0, time.perf_counter()
    while True:
        oc.csr_eval(off, m, cfg, votes, threads=threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": reps * gs / dt, "unit": "groups/s", "cores": threads, "kind": "port",
            "sample": f"{gs} groups of the same {kind} workload, C SoA restatement of "
                      f"majority.go/joint.go (oracle/quorum_oracle.c); {reps} passes on "
                      f"{threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warm-up steps (default 2000 x ~9 us for configs[1], 300 x "
                         "~0.2 ms for the CSR workloads: ~20-60 ms of work lets the clocks "
                         "settle; 20 warm-up steps measured 2-3 %% slow)")
    ap.add_argument("--groups", type=int, default=1 << 20, help="groups per GPU per step")
    ap.add_argument("--voters", type=int, default=5)
    ap.add_argument("--workload", default="fixed", choices=["fixed", "ragged", "joint"],
                    help="fixed = configs[1] (default); ragged = configs[2]; joint = configs[3]")
    ap.add_argument("--batches", type=int, default=16, help="distinct HBM-resident batches")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the steps rotate over")
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--graph", type=int, default=0,
                    help="launch the steps from a captured HIP graph of this many steps "
                         "(0 = direct launches); the remainder of K is launched directly")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal of the N > 1 path on fewer GPUs
            dist.init_process_group(args.backend)

    csr = args.workload != "fixed"
    if args.warmup is None:
        args.warmup = 300 if csr else 2000
    n, G, B, K, W = args.voters, args.groups, max(1, args.batches), args.steps, args.warmup
    S = max(1, args.streams)
    if csr:
        # configs[2]: 16M ragged groups per GPU; configs[3]: 64M joint groups over
        # 8 GPUs = 8M per GPU.  One batch is 0.7-1.3 GB (far beyond the 256 MB
        # MALL), so 2 resident batches suffice to keep consecutive steps apart.
        if args.groups == 1 << 20:
            G = (1 << 24) if args.workload == "ragged" else (1 << 23)
        B = min(B, 2)
    lib = _lib.load()
    main_stream = torch.cuda.current_stream(dev)
    msp = main_stream.cuda_stream
    streams = [torch.cuda.Stream(dev) for _ in range(S)]

    # B resident batches; global group numbers shard by rank (weak scaling)
    if csr:
        fn = lib.qb_dev_csr_committed_vote
        seed = {"ragged": 0x5EED0003, "joint": 0x5EED0004}[args.workload]
        groups = [batch.CsrGroups.synth(seed, args.workload, G, g_begin=(rank * B + b) * G,
                                        device=dev) for b in range(B)]
        slots = sum(int(g.off[-1].item()) for g in groups) / B
    else:
        fn = lib.qb_dev_fixed_committed_vote
        groups = [batch.FixedGroups.synth(SEED, n, G, g_begin=(rank * B + b) * G, device=dev)
                  for b in range(B)]
    outs = [(torch.empty(G, dtype=torch.int64, device=dev),
             torch.empty(G, dtype=torch.uint8, device=dev)) for _ in range(B)]
    # per step k: batch k % B on stream k % S (precomputed ctypes argument tuples)
    if csr:
        call_args = [[(G, g.max_slots, g.off.data_ptr(), g.match.data_ptr(), g.cfg.data_ptr(),
                       g.votes.data_ptr(), c.data_ptr(), v.data_ptr(), st.cuda_stream)
                      for g, (c, v) in zip(groups, outs)] for st in streams]
    else:
        call_args = [[(n, G, g.match.data_ptr(), g.voted.data_ptr(), g.granted.data_ptr(),
                       c.data_ptr(), v.data_ptr(), st.cuda_stream)
                      for g, (c, v) in zip(groups, outs)] for st in streams]
    torch.cuda.synchronize()

    def run_steps(count, fixed_batch=None):
        for st in streams:
            st.wait_stream(main_stream)
        for k in range(count):
            b = k % B if fixed_batch is None else fixed_batch
            rc = fn(*call_args[k % S][b])
            if rc:
                _lib.check(rc, "qb_dev_csr_committed_vote" if csr else "qb_dev_fixed_committed_vote")
        for st in streams:
            main_stream.wait_stream(st)

    graph = None
    if args.graph > 0:
        # one captured graph = args.graph consecutive steps over the same
        # batch/stream rotation as run_steps (forked from and joined back to
        # the capture stream), replayed on the main stream
        L = args.graph
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        with torch.cuda.graph(graph, stream=cap):
            for st in streams:
                st.wait_stream(cap)
            for k in range(L):
                rc = fn(*call_args[k % S][k % B])
                if rc:
                    _lib.check(rc, "capture")
            for st in streams:
                cap.wait_stream(st)
        torch.cuda.synchronize()
        eager_steps = run_steps

        def run_steps(count, fixed_batch=None):  # noqa: F811
            if fixed_batch is not None:
                return eager_steps(count, fixed_batch)
            for _ in range(count // L):
                graph.replay()
            if count % L:
                eager_steps(count % L)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    run_steps(W)
    ev = HipEvents(4)
    barrier()
    t0 = time.perf_counter()
    ev.record(ev.ev[0], msp)
    run_steps(K)
    ev.record(ev.ev[1], msp)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    avg_kernel_s = ev.elapsed_ms(0, 1) / 1e3 / K

    # MALL-warm single-batch rate (informational)
    run_steps(W, fixed_batch=0)
    torch.cuda.synchronize()
    tw = time.perf_counter()
    run_steps(K, fixed_batch=0)
    torch.cuda.synchronize()
    warm_elapsed = time.perf_counter() - tw
    ev.close()

    allgather_ms = None
    if world > 1:
        t = torch.tensor([elapsed, warm_elapsed, avg_kernel_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, warm_elapsed, avg_kernel_s = (float(x) for x in t.tolist())
        # node-wide result: all-gather one batch's commit (u64) and vote (u8)
        # vectors over RCCL (etcd_amd.shard)
        c, v = outs[0]
        for _ in range(3):
            allgather_results(c, v, world * G)
        barrier()
        ta = time.perf_counter()
        reps = 10
        for _ in range(reps):
            allgather_results(c, v, world * G)
        barrier()
        allgather_ms = (time.perf_counter() - ta) / reps * 1e3

    if rank == 0:
        total_groups = world * G * K
        value = total_groups / elapsed
        if csr:
            # off 4 + cfg 4 + votes 4 + match 8 per slot + commit 8 + vote 1
            bpg = 21 + 8 * slots / G
            key = f"csr_{args.workload}_G{G}"
            workload = {"ragged": "BASELINE configs[2]: 16M groups ragged 3-9 voters + learners "
                                  "(CSR offsets) per GPU, CommittedIndex + VoteResult",
                        "joint": "BASELINE configs[3]: JointConfig 5+5 CommittedIndex/VoteResult, "
                                 "8M groups per GPU (64M over 8 GPUs)"}[args.workload]
            cfg = {"workload": workload, "groups_per_gpu": G, "mean_slots": slots / G,
                   "layout": "CSR (off u32, cfg masks, votes, group-major match)"}
            ms = groups[0].max_slots
            kname = f"k_csr<{4 if ms <= 4 else 8 if ms <= 8 else 12 if ms <= 12 else 16},true,true>"
        else:
            bpg = bytes_per_group(n)
            key = f"fixed_n{n}_G{G}"
            cfg = {"workload": "BASELINE configs[1]: 1M groups x 5 voters CommittedIndex + "
                               "VoteResult, uint64 indexes, one MI355X per shard",
                   "groups_per_gpu": G, "voters": n, "layout": "fixed slot-major SoA"}
            kname = f"k_fixed<{n},2,true,true>"
        cfg.update({"batches_resident": B, "streams": S, "graph_steps": args.graph,
                    "parallelism": f"groups sharded by id over {world} GPU(s)"})
        achieved = bpg * G / avg_kernel_s / 1e9
        traffic = load_traffic(key)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "groups/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based splitmix64 spec, SURVEY.md §8d; HBM-resident)",
            "config": cfg,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kname,
                "bytes_per_group": bpg,
                "avg_kernel_us": avg_kernel_s * 1e6,
                "timing": (f"HIP events around the timed region on the launch streams; per-launch "
                           f"duration = region device time / K with {S} stream(s) overlapping "
                           f"consecutive launches"
                           + (f", launched from a HIP graph of {args.graph} steps"
                              if args.graph else "")),
            },
            "value_mall_warm": world * G * K / warm_elapsed,
            "allgather_ms": allgather_ms,
        }
        if world == 1 and not args.no_cpu_baseline and not csr:
            out["cpu_baseline"] = cpu_baseline(n, args.cpu_sample, args.cpu_seconds)
        elif world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_csr(args.workload, args.cpu_seconds)
        print(json.dumps(out), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
