"""Failure handling for bench.py's N-rank runs: every rank-local failure is
decided collectively, and nothing can wait forever.

A workload is a generator that ``yield``s a stage name before each group of
collectives (the "agreement points").  ``RankGuard.run`` resumes it stage by
stage; at every yield — and when the generator ends or raises — the ranks
all-reduce an error flag, so a failure on one rank (an exception in that
rank's local work) makes every rank leave the workload at the same point,
before any of them enters the next collective.  The rule the workloads keep:
no collective between two agreement points is preceded by fallible local
work on only some ranks, and no yield sits in a rank-dependent branch (every
rank yields the same stages in the same order).

Bounds on what agreement cannot catch (a hang inside a collective or a
kernel): a watchdog thread ends the process (exit 124) when one stage runs
past ``stage_timeout_s`` or the job past ``job_deadline_s``, after writing
the rank's stage to stderr and to ``$BENCH_STAGE_DIR/rank<r>.stage``; the
launcher (bench.spawn_ranks, or torchrun) then stops the other ranks.

Fault injection for the tests (``--inject-fail R:WORKLOAD:STAGE``,
``--inject-hang R:WORKLOAD:STAGE``): on rank R, the generator gets an
exception thrown in at that stage (a local failure), or the rank stops
making progress there (a local hang).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Generator, Optional


class WorkloadAborted(Exception):
    """Raised on every rank together when some rank failed a workload."""


def parse_inject(spec: Optional[str]):
    """'R:WORKLOAD:STAGE' -> (rank, workload, stage) or None."""
    if not spec:
        return None
    r, wl, st = spec.split(":", 2)
    return int(r), wl, st


class RankGuard:
    """One rank's stage tracker, failure agreement and watchdog.

    ``agree_fn(flag: int) -> int`` is the collective: the MAX of ``flag`` over
    the ranks (0 = ok, r + 1 = rank r failed); None at world 1.
    ``gather_fn(obj) -> list`` (optional) all-gathers one picklable object per
    rank: after a failure every rank learns each failing rank's stage and
    error."""

    def __init__(self, world: int, rank: int, agree_fn: Optional[Callable[[int], int]] = None,
                 stage_timeout_s: float = 600.0, job_deadline_s: float = 0.0,
                 stage_dir: Optional[str] = None, inject_fail=None, inject_hang=None,
                 exit_fn: Callable[[int], None] = os._exit,
                 gather_fn: Optional[Callable[[object], list]] = None):
        self.world, self.rank = world, rank
        self.agree_fn = agree_fn
        self.gather_fn = gather_fn
        self.stage_timeout_s = stage_timeout_s
        self.job_deadline = time.monotonic() + job_deadline_s if job_deadline_s > 0 else None
        self.stage_dir = stage_dir
        self.inject_fail, self.inject_hang = inject_fail, inject_hang
        self.exit_fn = exit_fn
        self.workload = "-"
        self.stage_name = "start"
        self._stage_deadline = time.monotonic() + stage_timeout_s
        self._stop = threading.Event()
        self._dog = None
        if stage_timeout_s > 0 or self.job_deadline is not None:
            self._dog = threading.Thread(target=self._watch, name="rankguard", daemon=True)
            self._dog.start()
        self.stage("start")

    # ------------------------------------------------------------ stages ---
    def stage(self, name: str, timeout_s: Optional[float] = None) -> None:
        """Enter a stage: reported on a timeout, its own deadline starts."""
        self.stage_name = name
        t = self.stage_timeout_s if timeout_s is None else timeout_s
        self._stage_deadline = time.monotonic() + t if t > 0 else float("inf")
        if self.stage_dir:
            try:
                with open(os.path.join(self.stage_dir, f"rank{self.rank}.stage"), "w") as f:
                    f.write(f"{self.workload}:{name} t={time.time():.1f}\n")
            except OSError:
                pass

    def where(self) -> str:
        return f"rank {self.rank}: workload {self.workload}, stage {self.stage_name}"

    def _watch(self) -> None:
        while not self._stop.wait(0.5):
            now = time.monotonic()
            why = None
            if now > self._stage_deadline:
                why = f"stage over its {self.stage_timeout_s:.0f} s limit"
            elif self.job_deadline is not None and now > self.job_deadline:
                why = "job deadline passed"
            if why:
                msg = f"bench.py watchdog: {self.where()}: {why}; exiting 124"
                print(msg, file=sys.stderr, flush=True)
                if self.stage_dir:
                    try:
                        with open(os.path.join(self.stage_dir, f"rank{self.rank}.stage"), "a") as f:
                            f.write(msg + "\n")
                    except OSError:
                        pass
                self.exit_fn(124)
                return

    def close(self) -> None:
        self._stop.set()

    # --------------------------------------------------------- agreement ---
    def agree(self, failed: bool) -> int:
        """Collective: 0 when no rank failed, else 1 + the highest failing
        rank.  Every rank must call it at the same agreement point."""
        flag = self.rank + 1 if failed else 0
        if self.world == 1 or self.agree_fn is None:
            return flag
        return int(self.agree_fn(flag))

    def _injected(self, stage: str, kind) -> bool:
        return kind is not None and kind[0] == self.rank and kind[1] == self.workload \
            and kind[2] == stage

    def _maybe_inject(self, stage: str) -> None:
        """Test hooks: the rank's local work up to agreement point ``stage``
        fails (an exception) or never finishes (a hang)."""
        if self._injected(stage, self.inject_hang):
            print(f"bench.py: injected hang at {self.where()}", file=sys.stderr, flush=True)
            while True:
                time.sleep(3600)
        if self._injected(stage, self.inject_fail):
            raise RuntimeError(f"injected failure before {self.workload}:{stage}")

    def run(self, workload: str, gen_fn: Callable[[], Generator]):
        """Run one workload generator under agreement (module docstring).
        Returns the generator's return value, or raises WorkloadAborted on
        every rank when any rank failed."""
        self.workload = workload
        self.stage("begin")
        err: Optional[BaseException] = None
        result = None
        gen = None
        stage = "setup"
        try:
            gen = gen_fn()
            self.stage("setup")
            self._maybe_inject("setup")
            stage = next(gen)
            self._maybe_inject(stage)
        except StopIteration as e:
            result, gen = e.value, None
        except Exception as ex:  # noqa: BLE001 — a rank-local failure, agreed below
            err = ex
        while True:
            if err is not None and gen is not None:
                gen.close()
                gen = None
            self.stage(f"agree@{stage}")
            bad = self.agree(err is not None)
            if bad:
                if gen is not None:
                    gen.close()
                mine = f"{type(err).__name__}: {err}" if err is not None else None
                if mine:
                    print(f"bench.py: {self.where()}: {mine}", file=sys.stderr, flush=True)
                # every rank learns who failed where (one more collective, all
                # ranks are here): [(rank, stage, error)] of the failing ranks
                rows = [(self.rank, stage, mine)]
                if self.gather_fn is not None and self.world > 1:
                    rows = self.gather_fn((self.rank, stage, mine))
                failures = [r for r in rows if r[2] is not None] or [(bad - 1, "?", "?")]
                raise WorkloadAborted("; ".join(f"rank {r} failed at stage {st!r} of {workload}: "
                                                f"{msg}" for r, st, msg in failures))
            if gen is None:
                self.stage("done")
                return result
            self.stage(stage)
            prev = stage
            try:
                stage = f"after {prev}"
                stage = next(gen)
                self._maybe_inject(stage)
            except StopIteration as e:
                result, gen = e.value, None
            except Exception as ex:  # noqa: BLE001 — agreed at the top of the loop
                err = ex
