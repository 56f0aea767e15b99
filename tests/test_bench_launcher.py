"""CPU tests of bench.py's multi-rank launcher and host-side helpers: the
``--gpus N`` spawn path (environment wiring, world agreement under a
launcher), the CPU-baseline host description, and the device-column
normalisation of the record routing (etcd_amd/shard.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from etcd_amd import shard  # noqa: E402


def test_launch_envs_wiring():
    envs = bench.launch_envs(4, {"PATH": "/x", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29123)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29123"
        assert e["PATH"] == "/x" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.launch_envs(1, {}, 1)[0]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_resolve_world():
    assert bench.resolve_world(1, {}) == (1, 0, 0, False)
    assert bench.resolve_world(8, {}) == (8, 0, 0, True)
    env = {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}
    assert bench.resolve_world(2, env) == (2, 1, 1, False)
    with pytest.raises(SystemExit, match="must agree"):
        bench.resolve_world(8, env)          # torchrun started 2 ranks, --gpus says 8
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_gpus_n_spawns_n_ranks_without_a_launcher():
    """``python bench.py --gpus 3`` with no torchrun starts three ranks, each
    with its own RANK / LOCAL_RANK, one WORLD_SIZE and one rendezvous."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3",
                          "--launch-check"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert sorted(r["rank"] for r in rows) == [0, 1, 2]
    assert sorted(r["local_rank"] for r in rows) == [0, 1, 2]
    assert {r["world"] for r in rows} == {3}
    assert len({r["master"] for r in rows}) == 1 and rows[0]["master"].startswith("127.0.0.1:")


def test_gpus_mismatch_under_launcher_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                          "--launch-check"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "must agree" in out.stderr


def test_host_cpu_info_fields():
    info = bench.host_cpu_info()
    assert info["affinity_cpus"] == len(os.sched_getaffinity(0)) >= 1
    assert info["logical_cpus"] == os.cpu_count()
    assert info["model"]                       # /proc/cpuinfo model name
    assert info["physical_cores"] is None or info["physical_cores"] >= 1
    assert 1 <= info["threads"] <= info["affinity_cpus"]


def test_route_columns_normalised_or_refused():
    """The device routing reads raw pointers: columns are converted to the
    layout it expects (any integer group dtype masked to uint32 bits, as the
    host path does; strided views made contiguous) or refused by dtype."""
    M = 10
    g64 = torch.arange(M, dtype=torch.int64) + (1 << 32)      # high bits masked off
    idx = torch.arange(2 * M, dtype=torch.int64)[::2]          # strided view
    cols = shard._device_columns({"group": g64, "flags": torch.zeros(M, dtype=torch.uint8),
                                  "index": idx, "term": torch.ones(M, dtype=torch.int64)})
    assert cols["group"].dtype == torch.int32 and cols["group"].tolist() == list(range(M))
    assert cols["index"].is_contiguous() and cols["index"].tolist() == list(range(0, 2 * M, 2))
    with pytest.raises(ValueError, match="flags"):
        shard._device_columns({"group": g64, "flags": torch.zeros(M, dtype=torch.int32),
                               "index": idx, "term": idx})
    with pytest.raises(ValueError, match="term"):
        shard._device_columns({"group": g64, "flags": torch.zeros(M, dtype=torch.uint8),
                               "index": idx, "term": idx.to(torch.int32)})
    with pytest.raises(ValueError, match="length"):
        shard._device_columns({"group": g64, "flags": torch.zeros(M + 1, dtype=torch.uint8),
                               "index": idx, "term": idx})
    with pytest.raises(ValueError, match="required"):
        shard._device_columns({"group": g64, "flags": torch.zeros(M, dtype=torch.uint8)})


def test_default_run_secondary_configs_wiring():
    """The default (configs[1], N = 1) run also measures configs[2]-[4] and
    the §8f rows: the flags and the bench_configs entry points next_rows()
    calls exist with the arguments it passes (the GPU side runs on the box)."""
    import inspect
    a = bench.parse_args([])
    assert a.workload == "fixed" and not a.no_others
    assert bench.parse_args(["--no-others"]).no_others
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs as bc
    for name, nargs in (("leader_config", 2), ("readindex_config", 2), ("wire_config", 2),
                        ("confchange_config", 2), ("wire_tracker_config", 2)):
        sig = inspect.signature(getattr(bc, name))
        required = [p for p in sig.parameters.values() if p.default is inspect.Parameter.empty]
        assert len(required) == nargs, name
    assert "rows" in inspect.signature(bc.wire_config).parameters
    assert callable(bench.next_rows) and callable(bench.run_other)


def _synthetic_line(n):
    """A default-run line of the shape bench.py prints at N ranks."""
    coll = lambda names: {c: {"ms": 1.0, "impl": "x", "ranks": n, "rccl_ranks": n}  # noqa: E731
                          for c in names}
    line = {k: 1 for k in bench.TOP_KEYS}
    line.update(n_gpus=n, value_per_rank=[1.0] * n, parity="bit-exact",
                roofline={k: 1 for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")})
    if n == 1:
        line["cpu_baseline"] = {}
    else:
        line["collectives"] = coll(bench.COLLECTIVES["fixed"])
        line["parity"] += "; node-wide all-gather bit-exact"
    line["other_configs"] = {}
    for wl in bench.OTHER_WORKLOADS:
        o = {"n_gpus": n, "value_per_rank": [1.0] * n, "parity": "bit-exact"}
        if n > 1:
            o["collectives"] = coll(bench.COLLECTIVES[wl])
            o["parity"] += "; node-wide: ..."
        line["other_configs"][wl] = o
    return line


@pytest.mark.parametrize("n", [1, 2, 8])
def test_line_shape_check(n):
    """bench.line_shape_errors accepts a complete line and names what a
    broken one lacks: at N > 1 every workload (configs[1]-[4]) must carry
    its timed collectives with their rank counts and a node-wide parity."""
    line = _synthetic_line(n)
    assert bench.line_shape_errors(line) == []
    bad = json.loads(json.dumps(line))
    del bad["other_configs"]["joint"]
    assert any("joint" in e for e in bench.line_shape_errors(bad))
    bad = json.loads(json.dumps(line))
    bad["value_per_rank"] = [1.0]
    assert (bench.line_shape_errors(bad) != []) == (n != 1)
    if n > 1:
        bad = json.loads(json.dumps(line))
        del bad["other_configs"]["tracker"]["collectives"]["route_records"]
        assert any("route_records" in e for e in bench.line_shape_errors(bad))
        bad = json.loads(json.dumps(line))
        bad["other_configs"]["tracker-csr"]["parity"] = "bit-exact"
        assert any("node-wide" in e for e in bench.line_shape_errors(bad))


COMMITTED_LINES = [
    "profiles/r04/multi/bench_n2_gloo_spawned.json",
    "profiles/r05/multi/bench_n8_gloo_spawned.json",
    "profiles/r05/multi/bench_n8_gloo_spawned_final.json",
]


@pytest.mark.parametrize("path", COMMITTED_LINES)
def test_committed_rehearsal_line_shape(path):
    """The committed `bench.py --gpus N --backend gloo` lines (N = 2, and the
    driver's N = 8 in round 5: N ranks spawned by bench.py on the one-GPU
    box, torch gloo collectives standing in for RCCL) have every key the
    N > 1 contract asks for."""
    with open(os.path.join(ROOT, path)) as f:
        line = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] in (2, 8)
    assert bench.line_shape_errors(line) == []


# ------------------------------------------------------- failure agreement ---
# bench.py's workloads run under tools/rankguard.py: a rank-local failure is
# decided by every rank together at the next agreement point, and a hang is
# bounded by each rank's watchdog and the launcher's deadline.  These run the
# real launcher and main loop over --fake-workloads (the workloads' stages and
# collectives on host tensors, gloo) at world 2.

def _fake_run(*extra, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    t0 = __import__("time").monotonic()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--fake-workloads", *extra], env=env, capture_output=True, text=True,
                         timeout=timeout)
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    return out, lines, __import__("time").monotonic() - t0


def test_fake_world2_run_reports_every_workload():
    out, lines, _ = _fake_run()
    assert out.returncode == 0, out.stderr[-2000:]
    assert len(lines) == 1
    line = lines[0]
    assert set(line["other_configs"]) == set(bench.OTHER_WORKLOADS)
    for wl, o in line["other_configs"].items():
        assert "error" not in o and "node-wide" in o["parity"], (wl, o)
        assert set(o["collectives"]) == set(bench.COLLECTIVES[wl])
    assert "failed_workloads" not in line


@pytest.mark.parametrize("inject", ["1:joint:setup", "1:joint:region", "0:tracker:region:end",
                                    "1:tracker-csr:allgather_results", "0:ragged:parity_agree"])
def test_injected_failure_every_rank_leaves_the_workload_together(inject):
    """An exception on one rank of a world-2 run: both ranks leave that
    workload at the same agreement point (nobody waits in a collective), the
    line names the failing rank and stage, every other workload still runs,
    and both ranks exit non-zero (4)."""
    out, lines, wall = _fake_run("--inject-fail", inject, "--stage-timeout-s", "60")
    assert out.returncode == 4, out.stderr[-2000:]
    r, wl, stage = inject.split(":", 2)
    line = lines[0]
    assert line["failed_workloads"] == [wl]
    err = line["other_configs"][wl]["error"]
    assert f"rank {r} failed at stage {stage!r}" in err and "injected failure" in err
    for other in bench.OTHER_WORKLOADS:
        if other != wl:
            assert "node-wide" in line["other_configs"][other]["parity"]
    assert wall < 120


def test_injected_headline_failure_prints_an_error_line():
    out, lines, _ = _fake_run("--inject-fail", "1:fixed:times", "--stage-timeout-s", "60")
    assert out.returncode == 4, out.stderr[-2000:]
    assert lines[0]["value"] is None and "rank 1 failed at stage 'times'" in lines[0]["error"]
    assert all("error" not in o for o in lines[0]["other_configs"].values())


def test_injected_hang_ends_within_the_stage_limit_and_names_the_stage():
    """A rank that stops making progress: the other rank's collective times
    out, the hung rank's watchdog exits 124, the launcher reports each
    rank's last stage — all within the stage limit plus the grace period."""
    out, _, wall = _fake_run("--inject-hang", "1:ragged:region", "--stage-timeout-s", "8",
                             "--deadline-s", "120")
    assert out.returncode != 0
    assert wall < 60, wall
    assert "ranks' last stages" in out.stderr
    assert "rank 1: ragged:" in out.stderr and "watchdog" in out.stderr


def test_job_deadline_terminates_the_ranks():
    """--deadline-s bounds the whole job whatever the stage limit."""
    out, _, wall = _fake_run("--inject-hang", "0:joint:setup", "--stage-timeout-s", "0",
                             "--deadline-s", "6")
    assert out.returncode != 0 and wall < 60, (out.returncode, wall)
    assert "job deadline passed" in out.stderr


def test_rankguard_world1_raises_local_failures_as_aborted():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from rankguard import RankGuard, WorkloadAborted

    def ok():
        yield "a"
        yield "b"
        return 7

    def boom():
        yield "a"
        raise ValueError("x")

    g = RankGuard(1, 0, stage_timeout_s=0)
    assert g.run("w", ok) == 7
    with pytest.raises(WorkloadAborted, match="rank 0 failed at stage 'after a' of w: ValueError"):
        g.run("w", boom)
    g.close()
