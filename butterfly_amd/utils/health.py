"""Failure detection and fault injection (detect and fail fast).

* HealthMonitor — every rank writes a heartbeat key into the job's TCPStore every `period`
  seconds; rank 0 checks them and, when one is older than `timeout`, publishes an abort key.
  Every rank's monitor thread watches that key and calls `on_failure(reason)` (default: log
  and terminate the process with exit code 75, so a launcher / torchrun restarts the job
  instead of every rank hanging in its next collective).
* StepWatchdog — arms a timer around each engine step; a step that outlives `timeout` (a hung
  collective, a GPU that stopped responding) dumps every thread's stack (faulthandler) and
  fires `on_failure`.
* ErrorPoller — a daemon thread polling a check (the native RCCL communicators' async errors)
  every second; on failure the registered abort hooks (`register_abort_hook`: abort every
  native communicator) run, bounded, before the process exits with 75.
* FaultInjector — BFLY_FAULT="rank:step:kind" (kind = hang | exit | nan) makes a chosen rank
  misbehave at a chosen step, so the detection paths are exercised by tests.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Callable, Optional

from . import flags
from .logging import get_logger

log = get_logger("health")


_abort_hooks: list = []


def register_abort_hook(fn: Callable[[], object]) -> None:
    """Run `fn` on the failure path before the process exits (parallel/rccl.abort_all: take
    the native RCCL communicators down so no kernel is left spinning on a dead peer)."""
    if fn not in _abort_hooks:
        _abort_hooks.append(fn)


def run_abort_hooks(timeout: float = 5.0) -> None:
    """Run the registered hooks on a daemon thread, bounded by `timeout`: an abort that itself
    hangs must not keep the process from exiting."""
    if not _abort_hooks:
        return

    def run():
        for fn in list(_abort_hooks):
            try:
                fn()
            except Exception as e:
                log.warning(f"abort hook {getattr(fn, '__name__', fn)} failed: {e!r}")

    t = threading.Thread(target=run, name="bfly-abort", daemon=True)
    t.start()
    t.join(timeout)
    if t.is_alive():
        log.error(f"abort hooks still running after {timeout}s; exiting anyway")


def _default_failure(reason: str) -> None:
    log.error(f"fatal: {reason}; terminating")
    faulthandler.dump_traceback(all_threads=True)
    sys.stderr.flush()
    run_abort_hooks()
    os._exit(75)


class ErrorPoller:
    """Polls `check() -> Optional[str]` every `period` seconds on a daemon thread and fires
    `on_failure(reason)` on the first non-None answer. Used for the native RCCL communicators'
    asynchronous errors (parallel/rccl.async_errors): the engine's own check_health runs only
    every 256 steps and never while a step is stuck in a collective; this thread does."""

    def __init__(self, check: Callable[[], Optional[str]], period: float = 1.0,
                 on_failure: Optional[Callable[[str], None]] = None, name: str = "bfly-errpoll"):
        self.check, self.period = check, period
        self.on_failure = on_failure or _default_failure
        self.name = name
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.failed: Optional[str] = None

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            try:
                reason = self.check()
            except Exception as e:   # library gone = teardown
                log.warning(f"{self.name} stopped: {e!r}")
                return
            if reason:
                self.failed = reason
                self.on_failure(reason)
                return

    def start(self) -> "ErrorPoller":
        if self.period > 0:
            self._thread = threading.Thread(target=self._run, name=self.name, daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=2 * self.period + 1)


class HealthMonitor:
    def __init__(self, store, rank: int, world: int, period: float = 5.0, timeout: float = 30.0,
                 on_failure: Optional[Callable[[str], None]] = None, prefix: str = "bfly/hb"):
        self.store, self.rank, self.world = store, rank, world
        self.period, self.timeout = period, timeout
        self.on_failure = on_failure or _default_failure
        self.prefix = prefix
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.failed: Optional[str] = None

    def beat(self) -> None:
        self.store.set(f"{self.prefix}/{self.rank}", repr(time.time()))

    def _check(self) -> Optional[str]:
        now = time.time()
        for r in range(self.world):
            try:
                v = self.store.get(f"{self.prefix}/{r}") if self.store.check([f"{self.prefix}/{r}"]) else None
            except Exception:
                v = None
            if v is None:
                continue
            age = now - float(v.decode() if isinstance(v, bytes) else v)
            if age > self.timeout:
                return f"rank {r} heartbeat is {age:.1f}s old (timeout {self.timeout}s)"
        return None

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self.beat()
                if self.rank == 0:
                    reason = self._check()
                    if reason:
                        self.store.set(f"{self.prefix}/abort", reason)
                if self.store.check([f"{self.prefix}/abort"]):
                    reason = self.store.get(f"{self.prefix}/abort").decode()
                    self.failed = reason
                    self.on_failure(reason)
                    return
            except Exception as e:  # store gone = the job is being torn down
                log.warning(f"health monitor stopped: {e!r}")
                return

    def start(self) -> "HealthMonitor":
        self.beat()
        self._thread = threading.Thread(target=self._run, name="bfly-health", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=2 * self.period)


class StepWatchdog:
    def __init__(self, timeout: float, on_failure: Optional[Callable[[str], None]] = None):
        self.timeout = timeout
        self.on_failure = on_failure or _default_failure
        self._timer: Optional[threading.Timer] = None
        self.fired: Optional[str] = None

    def arm(self, what: str = "step") -> None:
        self.disarm()
        if self.timeout > 0:
            def fire():
                self.fired = f"{what} exceeded {self.timeout}s"
                self.on_failure(self.fired)
            self._timer = threading.Timer(self.timeout, fire)
            self._timer.daemon = True
            self._timer.start()

    def disarm(self) -> None:
        if self._timer:
            self._timer.cancel()
            self._timer = None


class FaultInjector:
    def __init__(self, spec: Optional[str] = None):
        spec = spec if spec is not None else flags.get("BFLY_FAULT")
        self.rank = self.step = None
        self.kind = None
        # a restarted job (launch --max-restarts, BFLY_RESTART > 0) is the recovery path: the
        # fault is injected into the first attempt only
        if spec and os.environ.get("BFLY_RESTART", "0") not in ("", "0"):
            spec = None
        if spec:
            r, s, k = spec.split(":")
            self.rank, self.step, self.kind = int(r), int(s), k
            if k not in ("hang", "exit", "nan"):
                raise ValueError(f"unknown fault kind {k!r}")

    def maybe_inject(self, rank: int, step: int) -> Optional[str]:
        """Call once per step. Returns 'nan' when the caller should poison its output."""
        if self.kind is None or rank != self.rank or step != self.step:
            return None
        log.warning(f"injecting fault {self.kind!r} at step {step}")
        if self.kind == "exit":
            os._exit(13)
        if self.kind == "hang":
            while True:
                time.sleep(3600)
        return "nan"
