#!/usr/bin/env python3
"""Benchmark: raft groups quorum-evaluated per second on MI355X.

Workload (BASELINE.json configs[1]): 1M (2^20) raft groups x 5 voters per GPU,
CommittedIndex + VoteResult fused in one kernel, uint64 match indexes, FIXED
slot-major SoA layout.  One step = one pass of the hot path over one batch
of 2^20 groups.  ``--batches`` distinct batches (default 16, ~0.96 GB with
outputs) stay resident in HBM and are visited round-robin, so every step
streams its batch from HBM instead of the 256 MB Infinity Cache (the
MALL-warm single-batch rate is reported beside it as ``value_mall_warm``,
timed exactly as the headline).

Launch pipeline: consecutive steps are independent batches, so they are
issued round-robin on ``--streams`` HIP streams (default 2): the tail of one
launch overlaps the ramp of the next.  HIP events on the launch streams bracket
the timed region; the per-launch duration used for the roofline is the
region's device time / K.

``--workload ragged|joint`` runs BASELINE configs[2] / configs[3] (16M ragged
3-9-voter groups with learners / 8M JointConfig 5+5 groups per GPU, CSR
layout); ``--workload tracker|tracker-csr`` runs configs[4] (the streaming
MsgAppResp tracker step, 16M groups per GPU).  The default stays configs[1],
the metric's headline config.

Parity: after the timed region every workload checks its own output against
the C oracle (oracle/quorum_oracle.c) bit for bit and reports ``"parity"``;
a mismatch exits non-zero.

Multi-GPU: one process per GPU.  ``--gpus N`` with no launcher spawns the N
ranks itself (children get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; the
parent touches no GPU); under torchrun ``--gpus`` must equal WORLD_SIZE.
Groups shard by global group number (weak scaling, no collective in the
timed region).  For N > 1 the node-wide collectives are timed after the
region through the C ABI's RCCL communicator (etcd_amd/comm.py:
qb_dev_allgather_results, qb_dev_route_records — what a Go embedder binds),
and rank 0 checks the gathered vector against the oracle.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from etcd_amd import _lib  # noqa: E402
from etcd_amd.quorum import batch  # noqa: E402

METRIC = "raft groups quorum-evaluated/sec (1 and 8 GPUs) + % peak HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0x5EED0002      # 0x5EED0001 + config#
CSR_SEED = {"ragged": 0x5EED0003, "joint": 0x5EED0004}


def bytes_per_group(n: int) -> int:
    """Algorithmic bytes of the fused kernel per group:
    read match 8n + voted + granted masks, write commit 8 + vote 1."""
    mb = 1 if n <= 8 else 2
    return 8 * n + 2 * mb + 8 + 1


# ------------------------------------------------------------- launcher ---

def launch_envs(n: int, base: dict, port: int):
    """The environment of each of the n ranks ``--gpus n`` spawns (the
    variables torch.distributed.run sets; 127.0.0.1 rendezvous)."""
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool
        envs.append(e)
    return envs


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stage_report(stage_dir: str, n: int) -> str:
    """Each rank's last stage (tools/rankguard.py writes rank<r>.stage)."""
    rows = []
    for r in range(n):
        try:
            with open(os.path.join(stage_dir, f"rank{r}.stage")) as f:
                rows.append(f"  rank {r}: " + f.read().strip().replace("\n", " | "))
        except OSError:
            rows.append(f"  rank {r}: (no stage recorded)")
    return "\n".join(rows)


def spawn_ranks(n: int, argv, deadline_s: float = 0.0, grace_s: float = 30.0) -> int:
    """Start n child ranks of this same command (before any GPU call in this
    process: no exec, children are separate processes) and wait.  Returns 0,
    or the first non-zero exit code: the other ranks then get ``grace_s`` to
    finish on their own (every rank decides a workload's failure together
    and exits after rank 0 has printed its line) before they are terminated.
    With ``deadline_s`` > 0 every child still running at deadline_s + 60 s
    is terminated and 124 returned (each rank's own watchdog exits at
    deadline_s; this is the backstop).  On any failure each rank's last
    stage is printed to stderr."""
    import tempfile
    port = _free_port()
    stage_dir = tempfile.mkdtemp(prefix="bench_stages_")
    base = dict(os.environ, BENCH_STAGE_DIR=stage_dir)
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e)
             for e in launch_envs(n, base, port)]
    rc = 0
    t_end = time.monotonic() + deadline_s + 60.0 if deadline_s > 0 else None
    t_grace = None
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    t_grace = time.monotonic() + grace_s
            now = time.monotonic()
            if pending and ((t_grace is not None and now > t_grace)
                            or (t_end is not None and now > t_end)):
                if rc == 0:
                    rc = 124
                    print(f"bench.py: deadline ({deadline_s:.0f} s) passed; terminating "
                          f"{len(pending)} rank(s)", file=sys.stderr, flush=True)
                for q in pending:
                    q.terminate()
                for q in pending:
                    try:
                        q.wait(10)
                    except subprocess.TimeoutExpired:
                        q.kill()
                pending = []
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if rc != 0:
            print("bench.py: ranks' last stages:\n" + _stage_report(stage_dir, n),
                  file=sys.stderr, flush=True)
    return rc


def resolve_world(gpus: int, env) -> tuple:
    """(world, rank, local_rank, spawn): under a launcher WORLD_SIZE must
    equal --gpus; without one, --gpus > 1 means spawn."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} "
                             "ranks; they must agree")
        return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0")), False
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return gpus, 0, 0, gpus > 1


# --------------------------------------------------------------- timing ---

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


def timed_region(run, streams, K, barrier, name="region"):
    """K steps between barrier + synchronize.  Device time = from the earliest
    start event to the latest end event, one event pair per launch stream
    (no cross-stream hop inside the region: a fork + join around a 20-step
    region cost ~30 us of device time).  The start events are recorded after
    the barrier (device idle, so they stamp at once) and before t0; the wall
    clock stops when the host sees every stream's end event complete, then
    the device-wide synchronize runs (a torch.cuda.synchronize() costs ~20 us
    more than the event waits, 10 % of a 20-step region).
    A generator (``yield from``): agreement points (tools/rankguard.py)
    before each barrier, so a rank whose steps fail leaves together with the
    others.  Returns (wall seconds, device seconds per step)."""
    TS = len(streams)
    ev = HipEvents(2 * TS)
    yield name
    barrier()
    for s_, st in enumerate(streams):
        ev.record(ev.ev[s_], st.cuda_stream)
    t0 = time.perf_counter()
    run()
    for s_, st in enumerate(streams):
        ev.record(ev.ev[TS + s_], st.cuda_stream)
    for s_ in range(TS):
        ev.synchronize(TS + s_)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    yield name + ":end"
    barrier()
    starts = [0.0] + [ev.elapsed_ms(0, s_) for s_ in range(1, TS)]
    ends = [ev.elapsed_ms(0, TS + s_) for s_ in range(TS)]
    ev.close()
    return t1 - t0, (max(ends) - min(starts)) / 1e3 / K


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


# ---------------------------------------------------------- CPU baseline ---

def host_cpu_info() -> dict:
    """The host the CPU baseline runs on (core count, CPU model,
    thread count).  ``threads`` = the CPUs this process can actually run on:
    its affinity set, capped by the cgroup's CPU quota when one is set (the
    GPU box: 256 logical CPUs in the affinity set, a 16-CPU quota per GPU —
    256 threads there measured 2.5x slower than 16 on the tracker leg,
    quota throttling)."""
    info = {"logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "model": None, "physical_cores": None, "cgroup_cpu_quota": None}
    try:
        cores = set()
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and info["model"] is None:
                    info["model"] = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None:
                    cores.add((phys, core))
                    phys = core = None
        if phys is not None:
            cores.add((phys, core))
        info["physical_cores"] = len(cores) or None
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            info["cgroup_cpu_quota"] = float(q) / float(p)
    except (OSError, ValueError):
        pass
    q = info["cgroup_cpu_quota"]
    info["threads"] = max(1, min(info["affinity_cpus"], int(q))) if q else info["affinity_cpus"]
    return info


def oracle_threads(world: int) -> int:
    """Host threads for one rank's oracle checks: the CPUs this process may
    use, shared by the node's ranks (one process per GPU on one node)."""
    return max(1, host_cpu_info()["threads"] // max(1, world))


def _rate(fn, units, seconds):
    """units/s of fn() repeated for >= seconds (at least once)."""
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps * units / dt, reps


def cpu_baseline_eval(workload: str, n: int, seconds: float):
    """configs[1]-[3]: the oracle's two C restatements of the Go loop on a
    bounded 1M-group sample of the same workload, 1 thread and N = all host
    cores (BASELINE.md:21): the faithful one (Go-map MajorityConfig /
    JointConfig, ProgressMap and votes map, insertionSort; majority.go:126-210,
    joint.go:49-75) — the value — and the SoA one beside it."""
    from tests import oracle_c as oc
    info = host_cpu_info()
    N = info["threads"]
    gs = 1 << 20
    if workload == "fixed":
        match, vd, gr, _ = oc.gen_fixed(SEED, n, gs)
        maps = oc.faithful_maps(n, match, vd, gr)
        faithful = lambda th: oc.faithful_eval(maps, gs, threads=th)  # noqa: E731
        soa = lambda th: oc.fixed_eval(n, match, vd, gr, threads=th)  # noqa: E731
        what = f"{gs} groups x {n} voters"
    else:
        off, m, cfg, votes = oc.gen_csr(CSR_SEED[workload], workload, gs)
        maps = oc.faithful_csr_maps(off, m, cfg, votes)
        faithful = lambda th: oc.faithful_joint_eval(maps, gs, threads=th)  # noqa: E731
        soa = lambda th: oc.csr_eval(off, m, cfg, votes, threads=th)  # noqa: E731
        what = f"{gs} groups of the same {workload} workload"
    legs = {}
    for name, f in (("faithful", faithful), ("soa", soa)):
        for th in (1, N):
            legs[f"{name}_{th}t"] = _rate(lambda: f(th), gs, seconds / 4)[0]
    plumbing = None
    if workload == "fixed":
        # configs[0]: BenchmarkMajorityConfig_CommittedIndex (quorum/bench_test.go:
        # 24-40) — one n-voter config called in a loop, ns/op, faithful C
        # restatement on 1 thread (the device's ns per group is the line's
        # avg_kernel_us / groups)
        iters, lib = 1 << 20, oc.load()
        while True:
            t0 = time.perf_counter()
            lib.orc_bench_plumbing(n, iters, 0x5EED0001)
            dt = time.perf_counter() - t0
            if dt >= 0.5:
                break
            iters *= 4
        plumbing = {"voters": n, "cpu_ns_per_op": dt / iters * 1e9,
                    "reference": "raft/quorum/bench_test.go:24-40 (BASELINE configs[0])"}
    return {
        "value": legs[f"faithful_{N}t"], "unit": "groups/s", "cores": N, "kind": "port",
        "threads": N, "gomaxprocs_equivalent": N, "host": info, "legs": legs,
        "sample": (f"{what} (same synthetic spec); value = faithful C restatement of the Go loop "
                   f"(Go-map configs + AckedIndexer lookups + insertionSort, majority.go:126-210, "
                   f"joint.go:49-75) on {N} threads = every CPU the process may use (affinity "
                   f"{info['affinity_cpus']} logical CPUs, cgroup quota {info['cgroup_cpu_quota']}; "
                   f"GOMAXPROCS-equivalent {N}); legs: faithful and SoA restatements at 1 and {N} "
                   f"threads"),
        **({"configs0_plumbing": plumbing} if plumbing else {}),
    }


# ------------------------------------------------------------- tracker ---
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
TRACKER_STATE = ("match", "committed", "active", "stepdown_at")


# Skewed streams (--skew; VERDICT r4 "Next" 2): a massive multi-raft host's
# ticks have hot groups.  The same stream (one record per group per tick on
# average, E new entries per tick) with the records' groups drawn as
#   zipf         exact discrete Zipf(s = 1.1) over group ranks 1..G, ranks
#                mapped to groups by a fixed random permutation (the hottest
#                group gets ~11 % of the batch: ~1.9M records per 16M-record
#                tick, far above what raft lets one group receive);
#   zipf-capped  the same, with at most ZIPF_CAP records per group per tick:
#                a follower acks at most the MsgApps its leader has in flight,
#                MaxInflightMsgs = 4096 / 8 = 512 per follower in etcd
#                (server/etcdserver/raft.go:39, raft/raft.go:162), so 4 x 512
#                for a 5-voter group; the excess records are redrawn uniformly;
#   sb10 / sb30  10 % / 30 % of the records on the groups of ONE super-bucket
#                (chunks 0, 8, ..., 1016 of CH = 512 groups: the interleaved
#                super-bucket 0 of qb_bucket.h, 64K groups), the rest uniform.
SKEWS = ("none", "zipf", "zipf-capped", "sb10", "sb30")
ZIPF_S = 1.1
ZIPF_CAP = 4 * 512


def skewed_groups(G: int, M: int, skew: str, gen, dev, zipf=None) -> torch.Tensor:
    """M record groups (int32) of the given skew (SKEWS); ``zipf`` = the
    (cdf, permutation) pair shared by every batch of a stream."""
    if skew == "none":
        return torch.randint(0, G, (M,), generator=gen, device=dev, dtype=torch.int32)
    if skew.startswith("zipf"):
        cdf, perm = zipf
        u = torch.rand(M, generator=gen, device=dev, dtype=torch.float64)
        g = perm[torch.searchsorted(cdf, u).clamp_(max=G - 1)]
        if skew == "zipf-capped":
            # records past their group's ZIPF_CAP-th (in batch order) are redrawn
            order = torch.sort(g, stable=True).indices
            gs = g[order]
            first = torch.searchsorted(gs, gs, side="left")
            pos = torch.arange(M, device=dev) - first
            over = order[pos >= ZIPF_CAP]
            g[over] = torch.randint(0, G, (over.numel(),), generator=gen, device=dev)
        return g.to(torch.int32)
    frac = {"sb10": 0.1, "sb30": 0.3}[skew]
    g = torch.randint(0, G, (M,), generator=gen, device=dev, dtype=torch.int64)
    hot = torch.rand(M, generator=gen, device=dev) < frac
    nh = int(hot.sum().item())
    nchunks = min(128, ((G + 511) // 512 + 7) // 8)  # chunks 8j < NC of the first window
    c = 8 * torch.randint(0, nchunks, (nh,), generator=gen, device=dev)
    gg = c * 512 + torch.randint(0, 512, (nh,), generator=gen, device=dev)
    g[hot] = torch.minimum(gg, torch.tensor(G - 1, device=dev))
    return g.to(torch.int32)


def zipf_table(G: int, gen, dev):
    w = torch.arange(1, G + 1, dtype=torch.float64, device=dev).pow_(-ZIPF_S)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    return cdf, torch.randperm(G, generator=gen, device=dev)


# Group terms of the stream (--terms).  A raft group's term
# grows by one per election or leader transfer (raft.go:747-748, 785), so a
# massive multi-raft host holds groups of every age:
#   wide   (default) log-uniform over [1, 2^20): floor(2^(20 u)), u uniform —
#          about 45 % of the groups past 2045 (the compact record's term
#          field, qb_bucket.h), from fresh groups to ones a million elections
#          old;
#   small  every group at term 7 (the stream of rounds 1-5);
#   large  uniform over [20000, 2^20): every term past the field.
# 1 % of each tick's records carry the group's term - 1 (stale).
TRACKER_TERMS = ("wide", "small", "large")


def tracker_group_terms(G: int, terms: str, gen, dev) -> torch.Tensor:
    if terms == "small":
        return torch.full((G,), 7, dtype=torch.int64, device=dev)
    if terms == "large":
        return torch.randint(20000, 1 << 20, (G,), generator=gen, device=dev, dtype=torch.int64)
    u = torch.rand(G, generator=gen, device=dev, dtype=torch.float64)
    return torch.exp2(20.0 * u).floor_().clamp_(1, (1 << 20) - 1).to(torch.int64)


def tracker_batches(G, nb, last, n_slots_fn, gen, dev, gterm, skew="none"):
    """nb distinct streaming batches (device tensors); ``gterm``: the group
    terms (int64 [G])."""
    out = []
    zipf = zipf_table(G, gen, dev) if skew.startswith("zipf") else None
    for k in range(nb):
        group = skewed_groups(G, G, skew, gen, dev, zipf)
        slot = n_slots_fn(group, gen)
        lag = torch.randint(0, 96, (G,), generator=gen, device=dev, dtype=torch.int64)
        index = last[group.long()] + (k + 1) * TRACKER_E - lag
        t = gterm[group.long()]
        term = torch.where(torch.rand(G, generator=gen, device=dev) < 0.01, t - 1, t)
        out.append(batch.AppRespBatch(group, slot.to(torch.uint8), index, term))
    return out


def tracker_setup(G: int, nb: int, rank: int, dev, csr: bool, skew: str = "none",
                  terms: str = "wide"):
    """The configs[4] stream as the bench runs it: the leader state (after
    the initial maybeCommit, the leader's own match raised to the last of the
    nb * E entries it appended) and the nb device batches (``skew``: the
    records' group distribution, SKEWS; ``terms``: the group terms,
    TRACKER_TERMS).  Returns (tracker, batches, info).  tests/ replays
    exactly this stream on the oracle."""
    n = 5
    gen = torch.Generator(device=dev)
    gen.manual_seed(TRACKER_SEED + 7919 * rank)
    if csr:
        grp = batch.CsrGroups.synth(CSR_SEED["ragged"], "ragged", G, g_begin=rank * G, device=dev)
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
    gterm = tracker_group_terms(G, terms, gen, dev)
    tr.term.copy_(gterm)
    tr.commit_advance()
    batches = tracker_batches(G, nb, last, slots, gen, dev, gterm, skew=skew)
    big = float((gterm >= 2046).double().mean().item())
    if csr:
        tr.match[first] = last + nb * TRACKER_E   # the leader appended nb*E entries
    else:
        tr.match[0].copy_(last + nb * TRACKER_E)
    torch.cuda.synchronize(dev)
    return tr, batches, {"slots_mean": slots_mean, "voters_mean": voters_mean, "gen": gen,
                         "terms_past_field": big}


def tracker_host_state(tr, csr: bool, Gs: int, g0: int = 0):
    """Groups [g0, g0 + Gs) of a tracker's state as the oracle's numpy dict,
    rebased to local group 0 (off and cfg as well for the CSR layout)."""
    g0 = min(g0, tr.G)
    Gs = min(Gs, tr.G - g0)
    sl = slice(g0, g0 + Gs)
    if csr:
        off = tr.off[g0: g0 + Gs + 1].cpu().numpy().view(np.uint32).copy()
        a, e = int(off[0]), int(off[-1])
        off -= np.uint32(a)
        match = batch.as_u64(tr.match[a:e]).copy() if e > a else np.zeros(0, np.uint64)
        cfg = tr.cfg[sl].cpu().numpy().view(np.uint32).copy()
    else:
        off = cfg = None
        match = batch.as_u64(tr.match[:, sl]).copy()
    st = {"match": match, "committed": batch.as_u64(tr.committed[sl]).copy(),
          "active": tr.active[sl].cpu().numpy().view(np.uint16).copy(),
          "term": batch.as_u64(tr.term[sl]).copy(),
          "term_start": batch.as_u64(tr.term_start[sl]).copy(),
          "stepped_down": (tr.stepdown_at[sl] != -1).cpu().numpy().astype(np.uint8)}
    return off, cfg, st


def host_records(b, Gs: int, g0: int = 0):
    """The batch's records for groups [g0, g0 + Gs), in batch order, groups
    rebased to g0, as numpy."""
    g = b.group.long() & 0xFFFFFFFF
    keep = (g >= g0) & (g < g0 + Gs)
    return ((g[keep] - g0).to(torch.int32).cpu().numpy().view(np.uint32).copy(),
            b.flags[keep].cpu().numpy().copy(),
            batch.as_u64(b.index[keep]).copy(), batch.as_u64(b.term[keep]).copy())


def tracker_state_mismatches(tr, csr, st, Gs, g0: int = 0):
    """Fields where the device state of groups [g0, g0 + Gs) differs from the
    oracle's ``st``."""
    _, _, dev_st = tracker_host_state(tr, csr, Gs, g0)
    return [k for k in ("match", "committed", "active", "stepped_down")
            if not np.array_equal(dev_st[k], st[k])]


def parity_windows(G: int, Gs: int):
    """The tracker's parity windows: the whole shard when Gs >= G, else three
    windows of Gs / 3 groups (start, middle, end of the shard)."""
    if Gs >= G:
        return [(0, G)]
    w = max(1, Gs // 3)
    return [(0, w), ((G - w) // 2, w), (G - w, w)]


def tracker_cpu_baseline(seconds: float, csr: bool, terms: str = "wide"):
    """The oracle's sequential stepLeader restatement (one record at a time in
    batch order: term filter, MaybeUpdate, maybeCommit when updated;
    oracle/quorum_oracle.c appresp_range) on a bounded sample of the same
    stream: 1M groups, 8 consecutive 1M-record batches per pass, on 1 thread
    and on N = all host cores (groups partitioned over the threads, the batch
    stably partitioned by owning thread — exactly the sequential result)."""
    from tests import oracle_c as oc
    info = host_cpu_info()
    N = info["threads"]
    Gs, R, n = 1 << 20, 8, 5
    rng = np.random.default_rng(5)
    if csr:
        off, m0, cfg, _ = oc.gen_csr(CSR_SEED["ragged"], "ragged", Gs)
        sizes = np.diff(off.astype(np.int64))
        last = m0[off[:-1]].copy()            # slot 0 holds the leader's own match
        ts0 = last - np.uint64(64)
    else:
        m0, _, _, ts0 = oc.gen_fixed(TRACKER_SEED, n, Gs)
        last = m0[0].copy()
    if terms == "small":
        gterm = np.full(Gs, 7, np.uint64)
    elif terms == "large":
        gterm = rng.integers(20000, 1 << 20, size=Gs).astype(np.uint64)
    else:
        gterm = np.clip(np.floor(np.exp2(20.0 * rng.random(Gs))), 1, (1 << 20) - 1).astype(np.uint64)
    batches = []
    for k in range(R):
        grp = rng.integers(0, Gs, size=Gs).astype(np.uint32)
        if csr:
            slot = (1 + (rng.integers(0, 1 << 30, size=Gs) % (sizes[grp] - 1))).astype(np.uint8)
        else:
            slot = rng.integers(1, n, size=Gs).astype(np.uint8)
        lag = rng.integers(0, 96, size=Gs).astype(np.uint64)
        idx = last[grp] + np.uint64((k + 1) * TRACKER_E) - lag
        trm = np.where(rng.random(Gs) < 0.01, gterm[grp] - np.uint64(1), gterm[grp]).astype(np.uint64)
        batches.append((grp, slot, idx, trm))
    m_start = m0.copy()
    if csr:
        m_start[off[:-1]] = last + np.uint64(R * TRACKER_E)
    else:
        m_start[0] = last + np.uint64(R * TRACKER_E)

    def fresh():
        st = {"match": m_start.copy(), "active": np.zeros(Gs, np.uint16),
              "term": gterm.copy(), "term_start": ts0.copy(),
              "committed": np.zeros(Gs, np.uint64), "stepped_down": np.zeros(Gs, np.uint8)}
        if csr:
            oc.csr_commit_all(off, cfg, st["match"], ts0, st["committed"])
        else:
            oc.commit_all(n, st["match"], ts0, st["committed"])
        return st

    def rate(th, budget):
        busy, passes = 0.0, 0
        while busy < budget:
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

    rn, pn = rate(N, seconds / 2)
    r1, p1 = rate(1, seconds / 2)
    return {"value": rn, "unit": "group-steps/s", "cores": N, "kind": "port", "threads": N,
            "gomaxprocs_equivalent": N, "host": info,
            "legs": {f"sequential_{N}t": rn, "sequential_1t": r1},
            "sample": (f"{Gs} {'ragged CSR' if csr else '5-voter'} groups x {R} consecutive "
                       f"{Gs}-record batches of the same stream per pass, {pn} passes on {N} "
                       f"threads (every CPU the process may use: affinity {info['affinity_cpus']}, "
                       f"cgroup quota {info['cgroup_cpu_quota']}; GOMAXPROCS-equivalent {N}; "
                       f"groups partitioned, records stably partitioned by owner); 1 thread: "
                       f"{r1:.4g} group-steps/s over {p1} passes; group terms {terms} as the "
                       f"GPU stream; sequential C restatement of "
                       f"stepLeader's MsgAppResp path (oracle/quorum_oracle.c)"),
            "value_1thread": r1}


def tracker_parity(tr, csr, snaps, batches, threads):
    """The final device state of every parity window against the oracle's
    sequential replay of every batch the bench applied since the last
    restore (the nb batches in order), restricted to the window's groups.
    ``snaps``: [(g0, Gs, host state)] taken before the first batch."""
    from tests import oracle_c as oc
    bad = []
    for g0, Gs, (off, cfg, st) in snaps:
        for b in batches:
            rec = host_records(b, Gs, g0)
            if csr:
                oc.csr_appresp_sequential(off, cfg, rec, st, threads=threads)
            else:
                oc.appresp_sequential(5, len(st["committed"]), rec, st, threads=threads)
        bad += [f"{k} in [{g0}, {g0 + Gs})" for k in tracker_state_mismatches(tr, csr, st, Gs, g0)]
    return bad


def _timed(fn, barrier, warm=2, reps=5):
    """Mean wall ms of fn() over reps calls between barriers (after warm)."""
    out = None
    for _ in range(warm):
        out = fn()
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    barrier()
    return (time.perf_counter() - t0) / reps * 1e3, out


def _tracker_collectives(args, world, rank, dev, G, W, tr, batches, gen, restore, barrier):
    """configs[4]'s node-wide exchanges, timed after the region (SURVEY.md
    §8e): records arriving at any rank delivered to the owning shards
    (qb_dev_route_records), and the node-wide commit vector kept current by
    the changed-commit delta (qb_dev_allgather_changed) next to the full
    all-gather (qb_dev_allgather_results).  Node-wide checks: every record
    arrives at its owner (count, ownership and a checksum of the global group
    numbers over all ranks), and the delta-maintained vector equals a fresh
    full gather of every shard's committed vector after a real tick.
    A generator: an agreement point before every group of collectives."""
    total = world * G
    # routing: one batch of G records per rank with global group numbers
    b = batches[0]
    gl = torch.randint(0, total, (G,), generator=gen, device=dev, dtype=torch.int64)
    cols = {"group": gl.to(torch.int32), "flags": b.flags, "index": b.index, "term": b.term}
    yield "comm"
    route, route_impl = _router(args, dev)
    gather, gather_impl = _gather(args, dev)
    delta, delta_impl = _delta(args, dev)
    ranks = _rccl_ranks(args, world)
    yield "route_records"
    route_ms, got = _timed(lambda: route(cols, total), barrier)
    coll = {"route_records": {"ms": route_ms, "impl": route_impl, "ranks": world,
                              "rccl_ranks": ranks, "records_per_rank": G}}
    lg = got["group"].long() & 0xFFFFFFFF
    sums = torch.tensor([got["group"].numel(), int((lg + rank * G).sum().item()),
                         int(gl.sum().item()), G], dtype=torch.int64, device=dev)
    owned = bool((lg < G).all().item())
    yield "route_check"
    dist.all_reduce(sums)
    route_ok = _all_ok(owned, world, dev) and int(sums[0].item()) == int(sums[3].item()) \
        and int(sums[1].item()) == int(sums[2].item())
    # the changed-commit delta after a real tick, against a full gather
    vote0 = torch.zeros(G, dtype=torch.uint8, device=dev)
    adv = torch.zeros(G, dtype=torch.uint8, device=dev)
    restore()
    for k in range(W):
        tr.step(batches[k], reset_stats=False, rearm=False)
    torch.cuda.synchronize(dev)
    yield "allgather_results"
    commit_all, _ = gather(tr.committed, vote0, total)      # the vector before the tick
    commit_all = commit_all.to(dev).clone()
    tr.step(batches[W], advanced_out=adv, reset_stats=False, rearm=False)
    torch.cuda.synchronize(dev)
    yield "allgather_changed"
    delta_changed = delta(adv, tr.committed, total, commit_all)   # applied once: checked below
    full_ms, (full_c, _) = _timed(lambda: gather(tr.committed, vote0, total), barrier)
    same = torch.equal(commit_all, full_c.to(dev))
    scratch = commit_all.clone()
    yield "delta_check"
    delta_ok = _all_ok(same, world, dev)
    delta_ms, _ = _timed(lambda: delta(adv, tr.committed, total, scratch), barrier)
    coll["allgather_changed"] = {"ms": delta_ms, "impl": delta_impl, "ranks": world,
                                 "rccl_ranks": ranks, "changed_groups": delta_changed}
    coll["allgather_results"] = {"ms": full_ms, "impl": gather_impl, "ranks": world,
                                 "rccl_ranks": ranks, "bytes_received_per_rank": 9 * G * (world - 1)}
    note = ("node-wide: routing delivered every record to its owner (count, ownership, group "
            "checksum over all ranks)" if route_ok else "MISMATCH in the record routing")
    note += ("; the delta-maintained commit vector equals a full all-gather after a real tick"
             if delta_ok else "; MISMATCH between the changed-commit delta and a full all-gather")
    return route_ms, route_impl, delta_ms, delta_impl, delta_changed, coll, note


def tracker_main(args, world, rank, dev, barrier):
    """configs[4] (a generator run by RankGuard.run: agreement points before
    every collective)."""
    csr = args.workload == "tracker-csr"
    G = args.groups if args.groups != 1 << 20 else 1 << 24
    K = args.steps if args.steps != 1000 else 20
    W = args.warmup if args.warmup is not None else 4
    nb = W + K
    skew = getattr(args, "skew", "none") or "none"
    terms = getattr(args, "terms", "wide") or "wide"
    if nb > TRACKER_MAX_BATCHES:
        raise SystemExit(f"--workload {args.workload} keeps one distinct batch per step resident: "
                         f"--steps + --warmup must be <= {TRACKER_MAX_BATCHES}")
    tr, batches, info = tracker_setup(G, nb, rank, dev, csr, skew, terms)
    gen = info["gen"]
    snap = {k: getattr(tr, k).clone() for k in TRACKER_STATE}
    # the whole shard at N = 1; with N ranks sharing the node's CPUs, each
    # rank checks three windows (start, middle, end of its shard) of 2M
    # groups in all (the GPU suite checks the full 16M-group stream tick by
    # tick)
    tpg = args.tracker_parity_groups if args.tracker_parity_groups > 0 else (
        G if world == 1 else 1 << 21)
    windows = parity_windows(G, min(G, tpg))
    snaps = ([(g0, n_, tracker_host_state(tr, csr, n_, g0)) for g0, n_ in windows]
             if not args.no_parity else None)

    def restore():
        for k in TRACKER_STATE:
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
            # the Go caller's protocol: stepdown_at stays armed (the stream has
            # no higher-term record), no per-group re-arm write per tick
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

    def region():
        if pipe:  # the side stream's first bucketing starts inside the region
            for e in ev_a:
                e.record(main)
        for k in range(W, nb):
            step(batches[k])
    elapsed, step_s = yield from timed_region(region, [st], K, barrier)
    stats = tr.stats_dict()
    parity = None
    if snaps is not None:
        bad = tracker_parity(tr, csr, snaps, batches, oracle_threads(world))
        ng = sum(n_ for _, n_ in windows)
        where = ("the whole shard" if len(windows) == 1 else
                 "three windows of the shard: " + ", ".join(f"[{a}, {a + n_})" for a, n_ in windows))
        parity = (f"bit-exact {ng}/{ng} groups ({where}: match, committed, active, stepdown after "
                  f"all {nb} ticks vs the sequential C oracle)" if not bad
                  else f"MISMATCH in {bad} (after {nb} ticks)")
    route_ms = route_impl = delta_ms = delta_impl = delta_changed = None
    collectives = {}
    rate_local = G * K / elapsed
    yield "times"
    per_rank = _per_rank_values(rate_local, world)
    if world > 1:
        t = torch.tensor([elapsed, step_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_s = (float(x) for x in t.tolist())
        route_ms, route_impl, delta_ms, delta_impl, delta_changed, collectives, note = \
            yield from _tracker_collectives(args, world, rank, dev, G, W, tr, batches, gen,
                                            restore, barrier)
        parity = (parity or "") + "; " + note
    yield "parity_agree"
    parity = _agree(parity, world, dev)
    if rank != 0:
        return parity, None
    bpg = TRACKER_BYTES
    if csr:
        # record 21 + match RMW 16 + commit advance: off 4, cfg 4, the voters'
        # match 8 each (learners ack but do not count), term_start 8,
        # committed 8 read + 8 written
        bpg = 21 + 16 + 4 + 4 + 8 * info["voters_mean"] + 8 + 8 + 8
    key = f"tracker{'_csr' if csr else ''}_n5_G{G}" + ("" if terms == "small" else f"_{terms}")
    achieved = bpg * G / step_s / 1e9
    kern = ("memset, k_bk_scatter<true> (reserved regions), k_bk_split_compact, "
            + ("k_csr_apply<WMAX,8,false>, k_csr_apply_deferred, k_bk_slow<CsrLay<WMAX>>" if csr
               else "k_bk_apply<5,false>, k_bk_slow<FixedLay<5>>"))
    out = {
        "metric": METRIC + " — configs[4] streaming tracker: group-steps/s",
        "value": world * G * K / elapsed,
        "unit": "group-steps/s",
        "n_gpus": world, "rccl_ranks": _rccl_ranks(args, world), "steps": K, "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic streaming MsgAppResp batches (torch RNG on device, seeded per rank); "
                "leader state from the counter-based splitmix64 spec; HBM-resident",
        "config": {"workload": ("BASELINE configs[4]: streaming ProgressTracker, batched MsgAppResp "
                                "scatter-max + commit advance, 16M groups per GPU (128M over 8)"
                                + (" — ragged CSR groups (3-9 voters + 0-2 learners)" if csr
                                   else ", 5 voters")
                                + {"wide": "; group terms log-uniform over [1, 2^20) (raft terms "
                                           "of groups of every age, ~45 % past 2045)",
                                   "small": "; every group term 7",
                                   "large": "; group terms uniform over [20000, 2^20)"}[terms]),
                   "group_terms": terms, "terms_past_record_field": info["terms_past_field"],
                   "groups_per_gpu": G, "records_per_step": G, "new_entries_per_step": TRACKER_E,
                   "stale_term_fraction": 0.01, "mean_slots": info["slots_mean"],
                   "mean_voters": info["voters_mean"],
                   "skew": skew,
                   "pipelined_ticks": bool(pipe),
                   "parallelism": f"groups sharded by id over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic(key) if skew == "none" else None,
                     "kernel": f"{'qb_dev_csr_tracker_step' if csr else 'qb_dev_fixed_tracker_step'}"
                               f" (one step = {kern})",
                     "bytes_per_group": bpg, "avg_kernel_us": step_s * 1e6,
                     "timing": "HIP events around the K timed steps on the launch stream; "
                               "per-step device time = region / K (every kernel of the step)"
                               + ("; pipelined: tick k+1's bucketing (qb_dev_fixed_tracker_bucket) "
                                  "on a second stream while tick k is applied "
                                  "(qb_dev_fixed_tracker_apply), two workspaces" if pipe else "")},
        "parity": parity,
        "preroll_ms": preroll_ms, "preroll_steps": preroll_steps,
        "last_region_stats": {k: int(v) for k, v in stats.items()},
        "route_ms": route_ms, "route_impl": route_impl,
        "allgather_changed_ms": delta_ms, "allgather_changed_impl": delta_impl,
        "allgather_changed_groups": delta_changed,
        "collectives": collectives,
        "value_per_rank": per_rank,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = tracker_cpu_baseline(args.cpu_seconds, csr, terms)
    return parity, out


# ------------------------------------------------------ multi-GPU helpers ---

_COMM = []


def _comm(dev):
    """The C ABI's RCCL communicator (created once, after the timed region)."""
    if not _COMM:
        from etcd_amd.comm import RcclComm
        _COMM.append(RcclComm.from_process_group(dev))
    return _COMM[0]


def _rccl_ranks(args, world):
    return _COMM[0].world if _COMM else (world if args.backend == "nccl" and world > 1 else 0)


def _router(args, dev):
    if args.backend == "nccl":
        c = _comm(dev)
        first = [True]

        def route(cols, total):
            # the argument agreement (an all-reduce + a host sync) runs on the
            # first, untimed call only; every rank holds G records,
            # so the receive capacity is world x G without it
            a, first[0] = first[0], False
            return c.route_records(cols, total, out_cap=c.world * cols["group"].numel(), agree=a)
        return route, "qb_dev_route_records (RCCL C ABI; argument agreement on the first call only)"
    from etcd_amd.shard import route_records
    return route_records, f"etcd_amd.shard.route_records (torch {args.backend}, rehearsal)"


def _gather(args, dev):
    if args.backend == "nccl":
        c = _comm(dev)
        first = [True]

        def gather(cm, v, total):
            a, first[0] = first[0], False
            return c.allgather_results(cm, v, total, agree=a)
        return gather, "qb_dev_allgather_results (RCCL C ABI; argument agreement on the first call only)"
    from etcd_amd.shard import allgather_results
    return allgather_results, f"etcd_amd.shard.allgather_results (torch {args.backend}, rehearsal)"


def _delta(args, dev):
    if args.backend == "nccl":
        c = _comm(dev)
        first = [True]

        def delta(ch, cm, total, out):
            a, first[0] = first[0], False
            return c.allgather_changed(ch, cm, total, out, agree=a)
        return delta, "qb_dev_allgather_changed (RCCL C ABI; argument agreement on the first call only)"
    from etcd_amd.shard import allgather_changed
    return allgather_changed, f"etcd_amd.shard.allgather_changed (torch {args.backend}, rehearsal)"


def _agree(parity, world, dev):
    """Every rank's parity verdict (a mismatch anywhere is reported)."""
    if world == 1 or parity is None:
        return parity
    ok = torch.tensor([0 if "MISMATCH" in parity else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if "MISMATCH" in parity:
        return parity
    if int(ok.item()) == 0:
        return "MISMATCH on another rank"
    return parity + f" (every one of the {world} ranks)"


def _per_rank_values(x: float, world: int):
    """Every rank's own value (its groups / its own wall time), rank order."""
    if world == 1:
        return [float(x)]
    box = [None] * world
    dist.all_gather_object(box, float(x))
    return [float(y) for y in box]


def _all_ok(ok: bool, world: int, dev) -> bool:
    """True iff ``ok`` holds on every rank."""
    if world == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def _nodewide_eval_parity(args, world, rank, dev, G, B, n, gc, gv, c, v, threads):
    """The node-wide vectors after the all-gather: on every rank, its own
    slice equals its own outputs (which it checked bit-exact against the
    oracle over the whole shard); on rank 0, every rank's slice against the
    oracle over the first --parity-groups groups of that rank's batch 0 (the
    counter-based inputs regenerate any sub-range).  A generator: rank 0's
    oracle work is followed by an agreement point before the collective."""
    b0 = rank * G
    own = (torch.equal(gc[b0:b0 + G].to(dev), c) and torch.equal(gv[b0:b0 + G].to(dev), v))
    ok0 = True
    Gs = min(G, args.parity_groups)
    if rank == 0:
        hc = batch.as_u64(gc)
        hv = gv.cpu().numpy()
        for r in range(world):
            ec, ev_ = eval_oracle(eval_inputs_host(args.workload, n, Gs, (r * B) * G), threads)
            ok0 &= np.array_equal(hc[r * G:r * G + Gs], ec)
            ok0 &= np.array_equal(hv[r * G:r * G + Gs], ev_)
    yield "nodewide_parity"
    ok = _all_ok(own and ok0, world, dev)
    return (f"node-wide all-gather ({world} ranks) bit-exact: each rank's slice = its own checked "
            f"output, and rank 0 checked the first {Gs} groups of every rank's slice vs the oracle"
            if ok else "MISMATCH in the node-wide all-gather")


# ------------------------------------------------------- evaluation path ---

def eval_inputs_host(workload, n, G, g_begin):
    from tests import oracle_c as oc
    if workload == "fixed":
        match, vd, gr, _ = oc.gen_fixed(SEED, n, G, g_begin)
        return ("fixed", match, vd, gr)
    off, m, cfg, votes = oc.gen_csr(CSR_SEED[workload], workload, G, g_begin)
    return ("csr", off, m, cfg, votes)


def eval_oracle(inp, threads):
    from tests import oracle_c as oc
    if inp[0] == "fixed":
        _, match, vd, gr = inp
        return oc.fixed_eval(match.shape[0], match, vd, gr, threads=threads)
    _, off, m, cfg, votes = inp
    return oc.csr_eval(off, m, cfg, votes, threads=threads)


def eval_main(args, world, rank, dev, barrier):
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
        groups = [batch.CsrGroups.synth(CSR_SEED[args.workload], args.workload, G,
                                        g_begin=(rank * B + b) * G, device=dev) for b in range(B)]
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
    fname = "qb_dev_csr_committed_vote" if csr else "qb_dev_fixed_committed_vote"
    native = not csr and args.launcher == "native"
    if native:
        # configs[1]: the steps are enqueued from C (qb_dev_fixed_committed_vote_batches,
        # one ABI call per period of the batch/stream rotation) instead of one
        # ctypes call per launch
        import math

        class FixedBatch(C.Structure):
            _fields_ = [(f, C.c_void_p) for f in ("match", "voted", "granted", "commit_out",
                                                   "vote_out")]
        P = B * S // math.gcd(B, S)  # step k -> batch k % B on stream k % S

        def batch_table(pick):
            return (FixedBatch * P)(*[FixedBatch(groups[pick(k)].match.data_ptr(),
                                                 groups[pick(k)].voted.data_ptr(),
                                                 groups[pick(k)].granted.data_ptr(),
                                                 outs[pick(k)][0].data_ptr(),
                                                 outs[pick(k)][1].data_ptr()) for k in range(P)])
        tables = {None: batch_table(lambda k: k % B), 0: batch_table(lambda k: 0)}
        stream_arr = (C.c_void_p * S)(*[st.cuda_stream for st in streams])
        fnb = lib.qb_dev_fixed_committed_vote_batches

    def run_steps(count, fixed_batch=None, fork=True):
        # fork=False: the caller has synchronised the device, so the launch
        # streams need no cross-stream wait on the main stream (each such hop
        # costs device time: a fork + join around a 20-step region measured
        # ~30 us, 10.1 vs 8.6 us per launch)
        if fork:
            for st in streams:
                st.wait_stream(main_stream)
        if native:
            tab = tables[fixed_batch]
            full, rem = divmod(count, P)
            for c in [P] * full + ([rem] if rem else []):
                rc = fnb(n, G, c, tab, stream_arr, S)
                if rc:
                    _lib.check(rc, "qb_dev_fixed_committed_vote_batches")
        else:
            for k in range(count):
                b = k % B if fixed_batch is None else fixed_batch
                rc = fn(*call_args[k % S][b])
                if rc:
                    _lib.check(rc, fname)
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
    # (graph replays run on the main stream, forked inside the graph)
    tstreams = [main_stream] if graph is not None else streams
    elapsed, avg_kernel_s = yield from timed_region(lambda: run_steps(K, fork=graph is not None),
                                                    tstreams, K, barrier)

    # MALL-warm single-batch rate (informational): one batch (51 MB at
    # configs[1], inside the 256 MB MALL) re-read K times, timed exactly as
    # the region above (events on the launch streams, no fork/join)
    run_steps(W, fixed_batch=0)
    torch.cuda.synchronize()
    warm_elapsed, warm_kernel_s = yield from timed_region(
        lambda: run_steps(K, fixed_batch=0, fork=False), streams, K, barrier, "mall_warm")

    # parity: every resident batch's outputs (the last values written by the
    # timed steps; the MALL-warm pass rewrote batch 0 with the same result)
    # against the oracle on the same counter-based inputs
    parity = None
    threads = oracle_threads(world)
    if not args.no_parity:
        torch.cuda.synchronize()
        bad = 0
        for b in range(B):
            ec, ev_ = eval_oracle(eval_inputs_host(args.workload, n, G, (rank * B + b) * G), threads)
            c, v = outs[b]
            bad += int(not (np.array_equal(batch.as_u64(c), ec)
                            and np.array_equal(v.cpu().numpy(), ev_)))
        parity = (f"bit-exact {B}/{B} resident batches ({B * G} groups: CommittedIndex + "
                  f"VoteResult vs oracle/quorum_oracle.c)" if bad == 0
                  else f"MISMATCH in {bad}/{B} batches")

    allgather_ms = gather_impl = None
    collectives = {}
    rate_local = G * K / elapsed
    yield "times"
    per_rank = _per_rank_values(rate_local, world)
    if world > 1:
        t = torch.tensor([elapsed, warm_elapsed, avg_kernel_s, warm_kernel_s], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, warm_elapsed, avg_kernel_s, warm_kernel_s = (float(x) for x in t.tolist())
        # node-wide result: all-gather one batch's commit (u64) and vote (u8)
        # vectors, timed after the region
        yield "comm"
        gather, gather_impl = _gather(args, dev)
        c, v = outs[0]
        yield "allgather_results"
        for _ in range(3):
            gc, gv = gather(c, v, world * G)
        barrier()
        ta = time.perf_counter()
        reps = 10
        for _ in range(reps):
            gc, gv = gather(c, v, world * G)
        barrier()
        allgather_ms = (time.perf_counter() - ta) / reps * 1e3
        collectives["allgather_results"] = {
            "ms": allgather_ms, "impl": gather_impl, "ranks": world,
            "rccl_ranks": _rccl_ranks(args, world),
            "bytes_received_per_rank": 9 * G * (world - 1)}
        if not args.no_parity:
            parity = (parity or "") + "; " + (yield from _nodewide_eval_parity(
                args, world, rank, dev, G, B, n, gc, gv, c, v, threads))
    yield "parity_agree"
    parity = _agree(parity, world, dev)

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
                    "launcher": "native" if native else "python",
                    "parallelism": f"groups sharded by id over {world} GPU(s)"})
        achieved = bpg * G / avg_kernel_s / 1e9
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "groups/s",
            "n_gpus": world,
            "rccl_ranks": _rccl_ranks(args, world),
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
                "traffic": load_traffic(key),
                "kernel": kname,
                "bytes_per_group": bpg,
                "avg_kernel_us": avg_kernel_s * 1e6,
                "timing": (f"HIP events at the start and end of the timed region on each of the "
                           f"{len(tstreams)} launch stream(s); per-launch duration = (latest end - "
                           f"earliest start) / K, consecutive launches overlapping across the "
                           f"streams; wall clock from after the barrier to the host seeing every "
                           f"end event complete"
                           + (f", launched from a HIP graph of {args.graph} steps"
                              if args.graph else "")),
            },
            "parity": parity,
            "preroll_ms": preroll_ms,
            "preroll_steps": preroll_steps,
            "settle_probes": settle_probes,
            "settle_last_ratio": settle_ratio,
            "value_mall_warm": world * G * K / warm_elapsed,
            "mall_warm_kernel_us": warm_kernel_s * 1e6,
            "allgather_ms": allgather_ms,
            "allgather_impl": gather_impl,
            "collectives": collectives,
            "value_per_rank": per_rank,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_eval(args.workload, n, args.cpu_seconds)
        return parity, out
    return parity, None


def next_rows():
    """SURVEY §8f rows and configs[0] (tools/bench_configs.py, GPU side only:
    one device time per row) for the default run's line: the leader inbox
    step (4M groups), ReadIndex acks (4M leaders; local answers as
    ReadStates, the all-message form beside it), wire ingest (16M messages,
    group-row table), a conf change over 8M groups, the composed wire ->
    tracker tick in one call, FIXED and CSR (16M groups, 16M encoded
    MsgAppResp per tick; the chain's time beside it; decode + state parity in
    the row), and the configs[0]
    plumbing (the faithful C restatement's ns/op beside the device's ns per
    group).  Each row carries its own parity (round 5): the leader and
    ReadIndex workloads at 256K groups through every output form vs the C
    oracle, the wire decode of all 16M messages vs the C decoder, the conf
    change's whole result checked on the device, the composed rows' decode
    and state (the one call against the chain and the direct step, FIXED and
    CSR trackers); the GPU suite covers the rest (tests/test_gpu_leader.py,
    test_gpu_wire.py, test_gpu_confchange.py)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_configs as bc
    rows = []

    def report(name, groups, t, algo_bytes, extra=None):
        d = {"config": name, "per_launch_us": t * 1e6, "units_per_s": groups / t,
             "algo_bytes_per_unit": algo_bytes / groups, "achieved_GBs": algo_bytes / t / 1e9,
             "frac": algo_bytes / t / 1e9 / HBM_PEAK_GBS}
        d.update({k: v for k, v in (extra or {}).items() if k != "cpu_baseline"})
        rows.append(d)
    kw = {"reporter": report, "gpu_only": True}
    for name, fn in (("leader", lambda: bc.leader_config(1 << 22, 20, **kw)),
                     ("readindex", lambda: bc.readindex_config(1 << 22, 20, **kw)),
                     ("wire", lambda: bc.wire_config(1 << 24, 20, rows=True, **kw)),
                     ("confchange", lambda: bc.confchange_config(1 << 23, 20, **kw)),
                     ("wire-tracker", lambda: bc.wire_tracker_config(1 << 24, 10, **kw)),
                     ("wire-tracker-csr", lambda: bc.wire_tracker_config(1 << 24, 10, csr=True,
                                                                         **kw))):
        try:
            fn()
        except Exception as ex:  # reported; the headline stands
            rows.append({"config": name, "error": f"{type(ex).__name__}: {ex}"})
        torch.cuda.empty_cache()
    return rows


def other_summary(o2, p2):
    """The other_configs entry of one secondary workload's line."""
    r = o2["roofline"]
    d = {"workload": o2["config"]["workload"], "value": o2["value"], "unit": o2["unit"],
         "n_gpus": o2["n_gpus"], "steps": o2["steps"], "warmup": o2["warmup"],
         "ms_per_step": o2["ms_per_step"], "value_per_rank": o2.get("value_per_rank"),
         "roofline": {k: r.get(k) for k in ("achieved", "frac", "traffic", "bytes_per_group",
                                            "avg_kernel_us", "kernel")},
         "parity": p2}
    if o2.get("collectives"):
        d["collectives"] = o2["collectives"]
    return d


OTHER_WORKLOADS = ("ragged", "joint", "tracker", "tracker-csr")
# the node-wide collectives each workload times after its region at N > 1
COLLECTIVES = {"fixed": ("allgather_results",), "ragged": ("allgather_results",),
               "joint": ("allgather_results",),
               "tracker": ("route_records", "allgather_changed", "allgather_results"),
               "tracker-csr": ("route_records", "allgather_changed", "allgather_results")}
TOP_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline",
            "parity", "rccl_ranks", "value_per_rank")


def line_shape_errors(line: dict) -> list:
    """What the default run's JSON line lacks (tests/test_bench_launcher.py
    checks committed lines with it): the contract keys, the roofline and CPU
    baseline at N = 1, and at every N the four other BASELINE configs with a
    per-rank value each — plus, at N > 1, each workload's timed collectives
    (ms, implementation, rank count) and node-wide parity."""
    err = [f"missing {k}" for k in TOP_KEYS if k not in line]
    n = line.get("n_gpus", 0)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        if k not in line.get("roofline", {}):
            err.append(f"roofline.{k}")
    if n == 1 and "cpu_baseline" not in line:
        err.append("cpu_baseline at N = 1")
    if len(line.get("value_per_rank") or []) != n:
        err.append("value_per_rank: one value per rank")

    def colls(where, d, wl):
        if n <= 1:
            return
        for c in COLLECTIVES[wl]:
            e = (d.get("collectives") or {}).get(c)
            if not e or not all(k in e for k in ("ms", "impl", "ranks", "rccl_ranks")):
                err.append(f"{where}: collective {c} (ms, impl, ranks, rccl_ranks)")
            elif e["ranks"] != n or not e["ms"] or e["ms"] <= 0:
                err.append(f"{where}: collective {c} ranks / ms")
        if "node-wide" not in (d.get("parity") or ""):
            err.append(f"{where}: node-wide parity")
    colls("headline", line, "fixed")
    others = line.get("other_configs") or {}
    for wl in OTHER_WORKLOADS:
        o = others.get(wl)
        if not o or "error" in o:
            err.append(f"other_configs.{wl}: {o.get('error') if o else 'missing'}")
            continue
        if len(o.get("value_per_rank") or []) != n or o.get("n_gpus") != n:
            err.append(f"other_configs.{wl}: n_gpus / value_per_rank")
        if "MISMATCH" in (o.get("parity") or "MISMATCH"):
            err.append(f"other_configs.{wl}: parity")
        colls(f"other_configs.{wl}", o, wl)
    if "MISMATCH" in (line.get("parity") or ""):
        err.append("parity")
    return err


def run_other(args, world, rank, dev, barrier):
    """One secondary workload of the default run: the generator RankGuard.run
    drives (its parity, its JSON dict)."""
    if getattr(args, "fake_workloads", False):
        return fake_main(args, world, rank, dev, barrier)
    run = tracker_main if args.workload.startswith("tracker") else eval_main
    return run(args, world, rank, dev, barrier)


def fake_main(args, world, rank, dev, barrier):
    """CPU rehearsal of one workload (``--fake-workloads``; tests/
    test_bench_launcher.py): the stages and collectives of eval_main /
    tracker_main — region barriers, the per-rank values, a node-wide gather,
    the parity agreement — over tiny host tensors, so the failure agreement
    and the deadlines run without a GPU."""
    x = torch.arange(1 << 12, dtype=torch.int64)
    yield "region"
    barrier()
    t0 = time.perf_counter()
    y = int((x * 3).sum())
    elapsed = time.perf_counter() - t0 + 1e-6
    yield "region:end"
    barrier()
    parity = ("bit-exact (cpu rehearsal)" if y == 3 * ((1 << 12) - 1) * (1 << 11)
              else "MISMATCH (cpu rehearsal)")
    yield "times"
    per_rank = _per_rank_values(x.numel() / elapsed, world)
    coll = {}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        yield "allgather_results"
        out = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
        t0 = time.perf_counter()
        dist.all_gather(out, torch.full((4,), rank, dtype=torch.int64))
        ok = all(int(o[0]) == r for r, o in enumerate(out))
        for c in COLLECTIVES.get(args.workload, ("allgather_results",)):
            coll[c] = {"ms": (time.perf_counter() - t0) * 1e3 + 1e-3, "impl": "torch gloo (cpu)",
                       "ranks": world, "rccl_ranks": 0}
        parity += "; node-wide: all-gather of rank ids" + ("" if ok else " MISMATCH")
    yield "parity_agree"
    parity = _agree(parity, world, dev)
    if rank != 0:
        return parity, None
    return parity, {
        "metric": METRIC, "value": world * x.numel() / elapsed, "unit": "groups/s",
        "n_gpus": world, "rccl_ranks": 0, "steps": 1, "warmup": 0, "ms_per_step": elapsed * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "cpu rehearsal (--fake-workloads)",
        "config": {"workload": f"cpu rehearsal of {args.workload}"},
        "roofline": {k: None for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")},
        "parity": parity, "collectives": coll, "value_per_rank": per_rank}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a launcher, > 1 spawns them")
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
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline budget (split over its legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the post-region oracle check")
    ap.add_argument("--no-others", action="store_true",
                    help="the default (configs[1], N = 1) run skips the other BASELINE configs")
    ap.add_argument("--tracker-parity-groups", type=int, default=0,
                    help="tracker workloads: groups of the shard whose final state is checked "
                         "against the sequential oracle replay of every tick (0 = the whole shard "
                         "at N = 1, the first 2M groups of each rank's shard at N > 1)")
    ap.add_argument("--parity-groups", type=int, default=1 << 20,
                    help="N > 1, configs[1]-[3]: groups of every rank's slice of the node-wide "
                         "all-gather that rank 0 checks against the oracle")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--preroll-ms", type=float, default=300.0,
                    help="untimed clock-settle pre-roll before the warm-up steps (wall ms)")
    ap.add_argument("--graph", type=int, default=0,
                    help="launch the steps from a captured HIP graph of this many steps "
                         "(0 = direct launches); the remainder of K is launched directly")
    ap.add_argument("--launcher", default="native", choices=["native", "python"],
                    help="configs[1]: enqueue the steps from C (qb_dev_fixed_committed_vote_batches) "
                         "or with one ctypes call per launch")
    ap.add_argument("--lab-lib", default=None,
                    help="A/B lab runs: bind this build of libquorumbatch.so instead of the "
                         "in-tree one (etcd_amd._lib.use_lab_library)")
    ap.add_argument("--terms", default="wide", choices=list(TRACKER_TERMS),
                    help="configs[4] group terms: wide (log-uniform [1, 2^20), default), small "
                         "(all 7, rounds 1-5), large ([20000, 2^20))")
    ap.add_argument("--skew", default="none", choices=list(SKEWS),
                    help="tracker workloads: the records' group distribution (SKEWS: zipf = "
                         "Zipf(1.1) over groups, zipf-capped = at most 4 x 512 records per group, "
                         "sb10 / sb30 = 10 %% / 30 %% of the records on one super-bucket)")
    ap.add_argument("--deadline-s", type=float, default=1500.0,
                    help="job deadline: a rank still running after this long exits 124 naming "
                         "its stage (spawned ranks: the parent terminates them 60 s later); "
                         "0 = none")
    ap.add_argument("--stage-timeout-s", type=float, default=600.0,
                    help="one stage's limit (rank watchdog, and torch.distributed's collective "
                         "timeout); 0 = none")
    ap.add_argument("--inject-fail", default=None, help=argparse.SUPPRESS)   # R:WORKLOAD:STAGE
    ap.add_argument("--inject-hang", default=None, help=argparse.SUPPRESS)   # R:WORKLOAD:STAGE
    ap.add_argument("--fake-workloads", action="store_true", help=argparse.SUPPRESS)  # CPU tests
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def error_line(world: int, workload: str, err: str) -> dict:
    """The line rank 0 prints when the headline workload failed on some rank."""
    return {"metric": METRIC, "value": None, "unit": "groups/s", "n_gpus": world,
            "steps": None, "warmup": None, "ms_per_step": None, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": workload}, "roofline": None, "parity": None,
            "error": err}


def main():
    args = parse_args()
    world, rank, local, spawn = resolve_world(args.gpus, os.environ)
    if spawn:  # no GPU call has happened in this process
        sys.exit(spawn_ranks(world, sys.argv[1:], deadline_s=args.deadline_s))
    if args.launch_check:  # launcher wiring self-test (tests/test_bench_launcher.py)
        print(json.dumps({"rank": rank, "local_rank": local, "world": world,
                          "master": f"{os.environ.get('MASTER_ADDR')}:"
                                    f"{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from rankguard import RankGuard, WorkloadAborted, parse_inject
    if args.lab_lib:
        _lib.use_lab_library(args.lab_lib)
    fake = args.fake_workloads
    if fake:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
    if world > 1:
        import datetime
        kw = ({"timeout": datetime.timedelta(seconds=args.stage_timeout_s)}
              if args.stage_timeout_s > 0 else {})
        if args.backend == "nccl" and not fake:
            dist.init_process_group("nccl", device_id=dev, **kw)
        else:  # rehearsal of the N > 1 path on fewer GPUs (or none: --fake-workloads)
            dist.init_process_group(args.backend if not fake else "gloo", **kw)
    flag_dev = dev if (args.backend == "nccl" and not fake) else torch.device("cpu")

    def agree_fn(flag: int) -> int:
        t = torch.tensor([flag], dtype=torch.int32, device=flag_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    def gather_fn(obj):
        box = [None] * world
        dist.all_gather_object(box, obj)
        return box

    guard = RankGuard(world, rank, agree_fn if world > 1 else None, gather_fn=gather_fn,
                      stage_timeout_s=args.stage_timeout_s, job_deadline_s=args.deadline_s,
                      stage_dir=os.environ.get("BENCH_STAGE_DIR"),
                      inject_fail=parse_inject(args.inject_fail),
                      inject_hang=parse_inject(args.inject_hang))

    def barrier():
        if world > 1:
            dist.barrier()
        if not fake:
            torch.cuda.synchronize()

    failed = []
    try:
        parity, out = guard.run(args.workload, lambda: run_other(args, world, rank, dev, barrier))
    except WorkloadAborted as ex:
        parity, out = None, (error_line(world, args.workload, str(ex)) if rank == 0 else None)
        failed.append(args.workload)
    bad = parity is not None and "MISMATCH" in parity
    if args.workload == "fixed" and not args.no_others:
        # the other BASELINE configs, measured by the same command (so the
        # driver's own run backs them, at every N): configs[2] ragged,
        # configs[3] joint, configs[4] streaming tracker (fixed and ragged CSR
        # groups) — each at its full per-GPU size with its own warm-up, K = 20,
        # parity check and (N > 1) its node-wide collectives and checks.  Every
        # rank runs them (the collectives need all ranks); rank 0 reports.  A
        # failure on any rank is decided by every rank together at the next
        # agreement point (tools/rankguard.py): all ranks leave that workload,
        # the line names the error, the others still run.
        others = {}
        for wl in OTHER_WORKLOADS:
            sub = argparse.Namespace(**vars(args))
            sub.workload, sub.steps, sub.warmup, sub.no_cpu_baseline = wl, 20, None, True
            sub.preroll_ms, sub.settle_ms = min(args.preroll_ms, 200.0), min(args.settle_ms, 1000.0)
            sub.skew = "none"
            try:
                p2, o2 = guard.run(wl, lambda: run_other(sub, world, rank, dev, barrier))
            except WorkloadAborted as ex:  # every rank: reported in the line
                others[wl] = {"error": str(ex)}
                failed.append(wl)
                if not fake:
                    torch.cuda.empty_cache()
                continue
            bad |= p2 is not None and "MISMATCH" in p2
            if o2 is not None:
                others[wl] = other_summary(o2, p2)
            if not fake:
                torch.cuda.empty_cache()
        if out is not None:
            out["other_configs"] = others
            if world == 1 and not fake:
                guard.stage("next_rows")
                out["next_rows"] = next_rows()
    if out is not None:
        if failed:
            out["failed_workloads"] = failed
        print(json.dumps(out), flush=True)
    guard.stage("exit")
    for c in _COMM:
        c.close()
    if world > 1:
        guard.agree(False)  # no rank exits before rank 0 has printed the line
        dist.destroy_process_group()
    guard.close()
    if bad:
        sys.exit(3)
    if failed:
        sys.exit(4)


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException as ex:  # noqa: BLE001 — e.g. a collective timed out: no agreement left
        import traceback
        traceback.print_exc()
        print(f"bench.py: rank {os.environ.get('RANK', '0')}: {type(ex).__name__}: {ex}; "
              "exiting 5 (the process group cannot be trusted after this)", file=sys.stderr,
              flush=True)
        os._exit(5)
