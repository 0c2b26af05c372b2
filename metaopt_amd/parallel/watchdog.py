"""Rank-failure watchdog (SURVEY.md §5 "Failure detection / elastic recovery").

The reference detects a dead *worker* only through trial heartbeats: a reserved trial whose
heartbeat is older than ``worker.heartbeat`` becomes ``interrupted`` and reservable again
(reference src/orion/core/worker/experiment.py:217-232, src/orion/storage/legacy.py:206-217).
A device sweep adds a failure mode the reference never had: one process per GPU joined by
collectives, where a rank that dies (or a GPU that hangs) leaves every other rank blocked inside
an RCCL call forever.

``Watchdog`` is a daemon thread fed by ``beat(phase)`` from the sweep loop.  When no beat arrives
for ``timeout_s`` seconds it

1. records the stall (log + ``watchdog`` event in the JSONL log, if any);
2. runs the ``on_stall`` callbacks -- the sweep registers one on rank 0 that marks every
   in-flight trial ``interrupted`` in storage, so other workers (or a re-run of the same
   experiment) reserve them again, exactly as a lost heartbeat would after 120 s;
3. fails the process cleanly with ``exit_code`` (``os._exit``: the main thread is stuck in a
   collective and cannot unwind), so the launcher (``torchrun``) tears the job down instead of
   hanging until an outer time limit.

``exit_code=None`` only reports (tests, interactive use).  Beats are a single attribute store:
the hot loop pays nothing measurable.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
import time
from typing import Callable, List, Optional

log = logging.getLogger(__name__)


class Watchdog:
    def __init__(self, timeout_s: float, exit_code: Optional[int] = 75, poll_s: Optional[float] = None,
                 events=None, rank: int = 0):
        if timeout_s <= 0:
            raise ValueError("timeout_s must be positive")
        self.timeout_s = float(timeout_s)
        self.exit_code = exit_code
        self.poll_s = poll_s if poll_s is not None else min(1.0, self.timeout_s / 4)
        self.events = events
        self.rank = rank
        self.on_stall: List[Callable[[float, str], None]] = []
        self.fired = False
        self._last = time.monotonic()
        self._phase = "start"
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # -- fed by the sweep loop -------------------------------------------------------------------
    def beat(self, phase: str = "") -> None:
        self._last = time.monotonic()
        self._phase = phase

    # -- lifecycle ---------------------------------------------------------------------------------
    def start(self) -> "Watchdog":
        if self._thread is None:
            self._last = time.monotonic()
            self._thread = threading.Thread(target=self._run, name="mopt-watchdog", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(timeout=5 * self.poll_s + 1)
        self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # -- the thread ------------------------------------------------------------------------------
    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            stalled = time.monotonic() - self._last
            if stalled >= self.timeout_s:
                self._fire(stalled)
                return

    def _fire(self, stalled: float) -> None:
        self.fired = True
        phase = self._phase
        msg = (f"[watchdog] rank {self.rank}: no progress for {stalled:.1f}s "
               f"(last phase: {phase!r}); a peer rank or the GPU is presumed dead")
        log.error(msg)
        print(msg, file=sys.stderr, flush=True)
        if self.events is not None:
            try:
                self.events.emit("watchdog", stalled_s=round(stalled, 3), phase=phase)
                self.events.flush()
            except Exception:  # pragma: no cover - best effort while failing
                pass
        for cb in list(self.on_stall):
            try:
                cb(stalled, phase)
            except Exception as exc:  # the job is going down anyway; report and continue
                log.error("watchdog callback %r failed: %s", cb, exc)
        if self.exit_code is not None:
            sys.stderr.flush()
            sys.stdout.flush()
            os._exit(self.exit_code)
