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
        self.hip.hipEventSynchronize.argtypes = [C.c_void_p]
        self.ev = []
        for _ in range(count):
            e = C.c_void_p()
            assert self.hip.hipEventCreate(C.byref(e)) == 0
            self.ev.append(e)
        self.record = self.hip.hipEventRecord

    def synchronize(self, a: int):
        assert self.hip.hipEventSynchronize(self.ev[a]) == 0

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

# ------------------------------------------------------------------ tracker ---
# BASELINE configs[4]: "Streaming ProgressTracker: batched MsgAppResp
# scatter-max + commit advance, 128M groups x8 GPUs" = 16M 5-voter groups per
# GPU.  One step = one qb_dev_fixed_tracker_step over one batch of G records
# (one MsgAppResp per group on average, random arrival order, 1 % stale term)
# on HBM-resident leader state.  A live stream: the leader holds E new entries
# per step, batch k acknowledges last + (k+1)E - lag (lag < 96) for a random
# follower (slot 1..4) of a random group, so every step raises matches and
# advances commits (a replayed batch would leave the state unchanged after its
# first application).  Every step's batch is distinct and resident before the
# timed region (336 MB each).
TRACKER_E = 64
TRACKER_SEED = 0x5EED0005
TRACKER_MAX_BATCHES = 64
# SURVEY.md §8d per group-step: record 21 B (group 4, flags 1, index 8, term 8)
# + match RMW 16 B + commit advance 64 B (match 40 + term_start 8 + committed 8
# read, committed 8 written)
TRACKER_BYTES = 101


def tracker_batches(G, nb, last, n_slots_fn, gen, dev, seed_term=7):
    """nb distinct streaming batches (device tensors)."""
    out = []
    for k in range(nb):
        group = torch.randint(0, G, (G,), generator=gen, device=dev, dtype=torch.int32)
        slot = n_slots_fn(group, gen)
        lag = torch.randint(0, 96, (G,), generator=gen, device=dev, dtype=torch.int64)
        index = last[group.long()] + (k + 1) * TRACKER_E - lag
        term = torch.where(torch.rand(G, generator=gen, device=dev) < 0.01, seed_term - 1,
                           seed_term).to(torch.int64)
        out.append(batch.AppRespBatch(group, slot.to(torch.uint8), index, term))
    return out


def tracker_cpu_baseline(seconds: float, csr: bool):
    """The oracle's sequential stepLeader restatement (one record at a time in
    batch order: term filter, MaybeUpdate, maybeCommit when updated;
    oracle/quorum_oracle.c appresp_range) on a bounded sample of the same
    stream: 1M groups, 8 consecutive 1M-record batches per pass, groups
    partitioned over 16 host threads (each scans the batch for its own groups
    — exactly the sequential result) and on 1 thread."""
    from tests import oracle_c as oc
    threads = max(1, min(16, os.cpu_count() or 1))
    Gs, R, n = 1 << 20, 8, 5
    rng = np.random.default_rng(5)
    if csr:
        off, m0, cfg, _ = oc.gen_csr(0x5EED0003, "ragged", Gs)
        sizes = np.diff(off.astype(np.int64))
        last = m0[off[:-1]].copy()            # slot 0 holds the leader's own match
        ts0 = last - np.uint64(64)
    else:
        m0, _, _, ts0 = oc.gen_fixed(TRACKER_SEED, n, Gs)
        last = m0[0].copy()
    batches = []
    for k in range(R):
        grp = rng.integers(0, Gs, size=Gs).astype(np.uint32)
        if csr:
            slot = (1 + (rng.integers(0, 1 << 30, size=Gs) % (sizes[grp] - 1))).astype(np.uint8)
        else:
            slot = rng.integers(1, n, size=Gs).astype(np.uint8)
        lag = rng.integers(0, 96, size=Gs).astype(np.uint64)
        idx = last[grp] + np.uint64((k + 1) * TRACKER_E) - lag
        trm = np.where(rng.random(Gs) < 0.01, 6, 7).astype(np.uint64)
        batches.append((grp, slot, idx, trm))
    m_start = m0.copy()
    if csr:
        m_start[off[:-1]] = last + np.uint64(R * TRACKER_E)
    else:
        m_start[0] = last + np.uint64(R * TRACKER_E)

    def fresh():
        st = {"match": m_start.copy(), "active": np.zeros(Gs, np.uint16),
              "term": np.full(Gs, 7, np.uint64), "term_start": ts0.copy(),
              "committed": np.zeros(Gs, np.uint64), "stepped_down": np.zeros(Gs, np.uint8)}
        if csr:
            oc.csr_commit_all(off, cfg, st["match"], ts0, st["committed"])
        else:
            oc.commit_all(n, st["match"], ts0, st["committed"])
        return st

    def rate(th):
        busy, passes = 0.0, 0
        while busy < seconds:
            st = fresh()
            t = time.perf_counter()
            for b in batches:
                if csr:
                    oc.csr_appresp_sequential(off, cfg, b, st, threads=th)
                else:
                    oc.appresp_sequential(n, Gs, b, st, threads=th)
            busy += time.perf_counter() - t
            passes += 1
        return passes * R * Gs / busy, passes

    rn, pn = rate(threads)
    r1, p1 = rate(1)
    return {"value": rn, "unit": "group-steps/s", "cores": threads, "kind": "port",
            "sample": (f"{Gs} {'ragged CSR' if csr else '5-voter'} groups x {R} consecutive "
                       f"{Gs}-record batches of the same stream per pass, {pn} passes on {threads} "
                       f"threads (groups partitioned; GOMAXPROCS-equivalent {threads}); "
                       f"1 thread: {r1:.4g} group-steps/s over {p1} passes; sequential C "
                       f"restatement of stepLeader's MsgAppResp path (oracle/quorum_oracle.c)"),
            "value_1thread": r1}


def tracker_main(args, world, rank, dev):
    from etcd_amd.shard import route_records
    csr = args.workload == "tracker-csr"
    G = args.groups if args.groups != 1 << 20 else 1 << 24
    K = args.steps if args.steps != 1000 else 20
    W = args.warmup if args.warmup is not None else 4
    nb = W + K
    if nb > TRACKER_MAX_BATCHES:
        raise SystemExit(f"--workload {args.workload} keeps one distinct batch per step resident: "
                         f"--steps + --warmup must be <= {TRACKER_MAX_BATCHES}")
    n = 5
    gen = torch.Generator(device=dev)
    gen.manual_seed(TRACKER_SEED + 7919 * rank)
    if csr:
        grp = batch.CsrGroups.synth(0x5EED0003, "ragged", G, g_begin=rank * G, device=dev)
        tr = batch.CsrTracker(grp.off, grp.cfg, max_slots=grp.max_slots, device=dev)
        tr.match.copy_(grp.match[: tr.S])
        first = grp.off[:-1].long()
        last = tr.match[first].clone()        # slot 0: the leader's own match
        tr.term_start.copy_(last - 64)
        sizes = (grp.off[1:] - grp.off[:-1]).long()
        del grp

        def slots(group, g_):
            s_g = sizes[group.long()]
            r = torch.randint(0, 1 << 30, group.shape, generator=g_, device=dev)
            return 1 + r % (s_g - 1)
        slots_mean = float(sizes.float().mean())
        vm = (tr.cfg & 0xFFFF) | ((tr.cfg >> 16) & 0xFFFF)
        voters_mean = float(sum(((vm >> b) & 1).sum().item() for b in range(16))) / G
    else:
        tr = batch.FixedTracker(n, G, dev)
        fg = batch.FixedGroups.synth(TRACKER_SEED, n, G, g_begin=rank * G, device=dev,
                                     with_term_start=True)
        tr.match.copy_(fg.match)
        tr.term_start.copy_(fg.term_start)
        last = fg.match[0].clone()
        del fg

        def slots(group, g_):
            return torch.randint(1, n, group.shape, generator=g_, device=dev)
        slots_mean = voters_mean = float(n)
    tr.term.fill_(7)
    tr.commit_advance()
    batches = tracker_batches(G, nb, last, slots, gen, dev)
    if csr:
        tr.match[first] = last + nb * TRACKER_E   # the leader appended nb*E entries
    else:
        tr.match[0].copy_(last + nb * TRACKER_E)
    names = ("match", "committed", "active", "stepdown_at")
    snap = {k: getattr(tr, k).clone() for k in names}

    def restore():
        for k in names:
            getattr(tr, k).copy_(snap[k])

    pipe = args.pipeline and not csr
    if pipe:
        # Two ticks in flight: tick k+1's bucketing (records only) on a side
        # stream while tick k is applied on the launch stream
        # (qb_dev_fixed_tracker_bucket / _apply, include/quorum_batch.h).
        # apply(k) waits for bucket(k) (and, in stream order, apply(k-1));
        # bucket(k) waits for apply(k-2), the last reader of its workspace.
        wss = [tr.workspace(G), tr.workspace(G)]
        side = torch.cuda.Stream(dev)
        main = torch.cuda.current_stream(dev)
        ev_b = [torch.cuda.Event() for _ in range(2)]
        ev_a = [torch.cuda.Event() for _ in range(2)]
        for e in ev_a:
            e.record(main)
        nstep = [0]

    def step(b):
        if not pipe:
            tr.step(b, reset_stats=False, rearm=False)
            return
        j = nstep[0] & 1
        nstep[0] += 1
        side.wait_event(ev_a[j])
        tr.bucket(b, wss[j], stream=side)
        ev_b[j].record(side)
        main.wait_event(ev_b[j])
        tr.apply_bucketed(b, wss[j])
        ev_a[j].record(main)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # pre-roll: whole passes over the batches, state restored before each
    preroll_steps, tp = 0, time.perf_counter()
    while time.perf_counter() - tp < max(0.0, args.preroll_ms) / 1e3:
        restore()
        for b in batches:
            step(b)
        preroll_steps += nb
        torch.cuda.synchronize()
    preroll_ms = (time.perf_counter() - tp) * 1e3
    restore()
    for k in range(W):
        step(batches[k])
    tr.stats.zero_()
    st = torch.cuda.current_stream(dev)
    ev = HipEvents(2)
    barrier()
    ev.record(ev.ev[0], st.cuda_stream)
    if pipe:  # the side stream's first bucketing starts inside the region
        for e in ev_a:
            e.record(main)
    t0 = time.perf_counter()
    for k in range(W, nb):
        step(batches[k])
    ev.record(ev.ev[1], st.cuda_stream)
    ev.synchronize(1)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    barrier()
    elapsed = t1 - t0
    step_s = ev.elapsed_ms(0, 1) / 1e3 / K
    ev.close()
    stats = tr.stats_dict()
    route_ms = None
    if world > 1:
        t = torch.tensor([elapsed, step_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_s = (float(x) for x in t.tolist())
        # records arriving at arbitrary ranks: deliver one batch (G records per
        # rank, global group numbers over all shards) to the owning ranks
        # (etcd_amd.shard.route_records: RCCL all-to-all), timed apart
        b = batches[0]
        gl = torch.randint(0, world * G, (G,), generator=gen, device=dev, dtype=torch.int64)
        cols = {"group": gl.to(torch.int32), "flags": b.flags, "index": b.index, "term": b.term}
        for _ in range(2):
            route_records(cols, world * G)
        barrier()
        tr_ = time.perf_counter()
        for _ in range(5):
            route_records(cols, world * G)
        barrier()
        route_ms = (time.perf_counter() - tr_) / 5 * 1e3
    if rank != 0:
        return
    bpg = TRACKER_BYTES
    if csr:
        # record 21 + match RMW 16 + commit advance: off 4, cfg 4, the voters'
        # match 8 each (learners ack but do not count), term_start 8,
        # committed 8 read + 8 written
        bpg = 21 + 16 + 4 + 4 + 8 * voters_mean + 8 + 8 + 8
    key = f"tracker{'_csr' if csr else ''}_n5_G{G}"
    achieved = bpg * G / step_s / 1e9
    kern = ("k_bk_hist, k_scan_local, k_bk_sums_parts, k_bk_scatter, k_bk_split, "
            + ("k_csr_apply<WMAX,8,false>, k_csr_apply_deferred, k_bk_slow<CsrLay<WMAX>>" if csr
               else "k_bk_apply<5,false>, k_bk_slow<FixedLay<5>>"))
    out = {
        "metric": METRIC + " — configs[4] streaming tracker: group-steps/s",
        "value": world * G * K / elapsed,
        "unit": "group-steps/s",
        "n_gpus": world, "steps": K, "warmup": W, "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic streaming MsgAppResp batches (torch RNG on device, seeded per rank); "
                "leader state from the counter-based splitmix64 spec; HBM-resident",
        "config": {"workload": ("BASELINE configs[4]: streaming ProgressTracker, batched MsgAppResp "
                                "scatter-max + commit advance, 16M groups per GPU (128M over 8)"
                                + (" — ragged CSR groups (3-9 voters + 0-2 learners)" if csr
                                   else ", 5 voters")),
                   "groups_per_gpu": G, "records_per_step": G, "new_entries_per_step": TRACKER_E,
                   "stale_term_fraction": 0.01, "mean_slots": slots_mean,
                   "mean_voters": voters_mean,
                   "pipelined_ticks": bool(pipe),
                   "parallelism": f"groups sharded by id over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(key),
                     "kernel": f"{'qb_dev_csr_tracker_step' if csr else 'qb_dev_fixed_tracker_step'}"
                               f" (one step = {kern})",
                     "bytes_per_group": bpg, "avg_kernel_us": step_s * 1e6,
                     "timing": "HIP events around the K timed steps on the launch stream; "
                               "per-step device time = region / K (every kernel of the step)"
                               + ("; pipelined: tick k+1's bucketing (qb_dev_fixed_tracker_bucket) "
                                  "on a second stream while tick k is applied "
                                  "(qb_dev_fixed_tracker_apply), two workspaces" if pipe else "")},
        "preroll_ms": preroll_ms, "preroll_steps": preroll_steps,
        "last_region_stats": {k: int(v) for k, v in stats.items()},
        "route_ms": route_ms,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = tracker_cpu_baseline(args.cpu_seconds, csr)
    print(json.dumps(out), flush=True)



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
    ap.add_argument("--settle-ms", type=float, default=2000.0,
                    help="configs[1]-[3]: at most this long, untimed 64-step probes before the "
                         "timed region until one runs within 10 %% of the pre-roll's fastest")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="tracker workload: 1 = overlap tick k+1's bucketing with tick k's apply "
                         "on two streams (bucket / apply entry points; measured 5 %% slower: "
                         "the concurrent kernels contend); 0 = one qb_dev_fixed_tracker_step "
                         "per tick (default)")
    ap.add_argument("--workload", default="fixed",
                    choices=["fixed", "ragged", "joint", "tracker", "tracker-csr"],
                    help="fixed = configs[1] (default); ragged = configs[2]; joint = configs[3]; "
                         "tracker = configs[4] (streaming MsgAppResp step, FIXED 5 voters); "
                         "tracker-csr = the same stream over ragged CSR groups")
    ap.add_argument("--batches", type=int, default=16, help="distinct HBM-resident batches")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the steps rotate over")
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--preroll-ms", type=float, default=300.0,
                    help="untimed clock-settle pre-roll before the warm-up steps (wall ms)")
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

    if args.workload.startswith("tracker"):
        tracker_main(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return
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

    def run_steps(count, fixed_batch=None, fork=True):
        # fork=False: the caller has synchronised the device, so the launch
        # streams need no cross-stream wait on the main stream (each such hop
        # costs device time: a fork + join around a 20-step region measured
        # ~30 us, 10.1 vs 8.6 us per launch)
        if fork:
            for st in streams:
                st.wait_stream(main_stream)
        for k in range(count):
            b = k % B if fixed_batch is None else fixed_batch
            rc = fn(*call_args[k % S][b])
            if rc:
                _lib.check(rc, "qb_dev_csr_committed_vote" if csr else "qb_dev_fixed_committed_vote")
        if fork:
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

        def run_steps(count, fixed_batch=None, fork=True):  # noqa: F811
            if fixed_batch is not None:
                return eager_steps(count, fixed_batch, fork)
            for _ in range(count // L):
                graph.replay()
            if count % L:
                eager_steps(count % L)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # Clock-settle pre-roll: untimed steps of the same workload until at least
    # --preroll-ms of wall time has passed, whatever --warmup is (a 5-step
    # warm-up leaves the clocks ramping: the round-1 driver line measured
    # 9.85 us per launch against 8.6 us settled).  Then the W warm-up steps.
    preroll_steps, tp = 0, time.perf_counter()
    preroll_s = max(0.0, args.preroll_ms) / 1e3
    best64 = float("inf")  # fastest 64-step chunk (wall, synchronised)
    while time.perf_counter() - tp < preroll_s:
        tc = time.perf_counter()
        run_steps(64)
        preroll_steps += 64
        torch.cuda.synchronize()
        best64 = min(best64, time.perf_counter() - tc)
    preroll_ms = (time.perf_counter() - tp) * 1e3
    run_steps(W)
    # Settle guard (untimed): one box ran the timed region and the MALL-warm
    # pass after it at 0.6x the pre-roll's rate (a transient slowdown that the
    # pre-roll had not seen).  Before the region, 64-step probes are run until
    # one is within 10 % of the pre-roll's fastest chunk (at most --settle-ms);
    # the probes and their last ratio are reported.
    settle_probes, settle_ratio, ts_ = 0, None, time.perf_counter()
    if best64 < float("inf"):
        while time.perf_counter() - ts_ < max(0.0, args.settle_ms) / 1e3:
            torch.cuda.synchronize()
            tc = time.perf_counter()
            run_steps(64)
            torch.cuda.synchronize()
            settle_probes += 1
            settle_ratio = (time.perf_counter() - tc) / best64
            if settle_ratio <= 1.10:
                break
    # Timed region: K steps between barrier + synchronize.  Device time = from
    # the earliest start event to the latest end event, one event pair per
    # launch stream (no cross-stream hop inside the region: a fork + join
    # around a 20-step region cost ~30 us of device time).  The start events
    # are recorded after the barrier (device idle, so they stamp at once) and
    # before t0; the wall clock stops when the host sees every stream's end
    # event complete (hipEventSynchronize: all K steps are done), then the
    # device-wide synchronize runs (tools/lab/sync_overhead.py: a
    # torch.cuda.synchronize() costs ~20 us more than the event waits, a fixed
    # cost that is 10 % of a 20-step region).
    # (graph replays run on the main stream, forked inside the graph)
    tstreams = [main_stream] if graph is not None else streams
    TS = len(tstreams)
    ev = HipEvents(2 * TS)
    barrier()
    for s_, st in enumerate(tstreams):
        ev.record(ev.ev[s_], st.cuda_stream)
    t0 = time.perf_counter()
    run_steps(K, fork=graph is not None)
    for s_, st in enumerate(tstreams):
        ev.record(ev.ev[TS + s_], st.cuda_stream)
    for s_ in range(TS):
        ev.synchronize(TS + s_)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    barrier()
    elapsed = t1 - t0
    starts = [0.0] + [ev.elapsed_ms(0, s_) for s_ in range(1, TS)]
    ends = [ev.elapsed_ms(0, TS + s_) for s_ in range(TS)]
    avg_kernel_s = (max(ends) - min(starts)) / 1e3 / K

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
            kname = (f"k_fixed_lds<{n},{4 if n <= 5 else 2},true>" if n <= 8
                     else f"k_fixed<{n},2,true,true>")
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
                "timing": (f"HIP events at the start and end of the timed region on each of the "
                           f"{S} launch stream(s); per-launch duration = (latest end - earliest "
                           f"start) / K, consecutive launches overlapping across the streams; "
                           f"wall clock from after the barrier to the host seeing every end "
                           f"event complete"
                           + (f", launched from a HIP graph of {args.graph} steps"
                              if args.graph else "")),
            },
            "preroll_ms": preroll_ms,
            "preroll_steps": preroll_steps,
            "settle_probes": settle_probes,
            "settle_last_ratio": settle_ratio,
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
