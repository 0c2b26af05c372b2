"""Heartbeats of running trials.

Behaviour contract (reference ``src/orion/core/worker/trial_pacemaker.py:14-52``): while a trial
runs, its ``heartbeat`` in storage is refreshed every ``wait_time`` seconds; the refreshes stop
once the trial is completed / interrupted / suspended / broken, or when a refresh fails (the trial
was declared lost and taken over by another worker).

Structure: one dispatcher thread serves every pacemaker of the process from a deadline heap and
hands due beats to a few worker threads -- a study holding many reserved trials
(``client/study.py``) costs at most five threads, not one per trial, and one stalled storage call
holds up only its own trial's heartbeat.
:class:`TrialPacemaker` is a handle on one entry: ``start`` schedules it, ``stop`` cancels it
and returns once no beat of it is running, ``stopped`` is set when it ends for any reason.
"""
from __future__ import annotations

import collections
import heapq
import itertools
import logging
import threading
import time

log = logging.getLogger(__name__)

STOPPED_STATUS = {"completed", "interrupted", "suspended", "broken"}


class _Scheduler:
    """Deadline heap of pacemakers.  One daemon dispatcher thread pops due entries; the beats
    themselves (storage round trips) run on a few daemon worker threads, so one slow or stalled
    storage call (a contended PickledDB lock, a slow MongoDB) delays only its own trial's beat,
    never the other trials' -- their heartbeats stay fresh.  Threads start on first use and end
    when idle."""

    MAX_WORKERS = 4
    IDLE_EXIT_S = 1.0

    def __init__(self):
        self._cv = threading.Condition()
        self._heap = []                     # (due, seq, pacemaker)
        self._seq = itertools.count()
        self._thread = None                 # dispatcher
        self._ready = collections.deque()   # due pacemakers waiting for a worker
        self._running = set()               # pacemakers whose beat is in progress
        self._workers = 0
        self._idle = 0

    def add(self, pm, due):
        with self._cv:
            self._push(pm, due)

    def _push(self, pm, due):
        """Schedule ``pm`` at ``due`` (caller holds the lock); (re)start the dispatcher if it
        has exited, so a beat re-queued after a long storage call is never orphaned."""
        heapq.heappush(self._heap, (due, next(self._seq), pm))
        if self._thread is None or not self._thread.is_alive():
            self._thread = threading.Thread(target=self._dispatch, name="mopt-heartbeats",
                                            daemon=True)
            self._thread.start()
        self._cv.notify_all()

    def wait_idle(self, pm):
        """Block until ``pm`` is not being beaten (its entry may still sit in the heap or the
        ready queue, where it is skipped once ``pm.stopped`` is set)."""
        with self._cv:
            while pm in self._running:
                self._cv.wait(0.05)

    def _dispatch(self):
        while True:
            with self._cv:
                while self._heap and self._heap[0][2].stopped.is_set():
                    heapq.heappop(self._heap)              # cancelled entries
                if not self._heap:
                    self._cv.wait(self.IDLE_EXIT_S)
                    # exit only when nothing can come back: no entry queued and no beat in
                    # progress (a running beat re-queues itself when it finishes)
                    if not self._heap and not self._running and not self._ready:
                        self._thread = None
                        return                              # idle: the next add restarts it
                    continue
                due = self._heap[0][0]
                now = time.monotonic()
                if due > now:
                    self._cv.wait(due - now)
                    continue
                _, _, pm = heapq.heappop(self._heap)
                self._running.add(pm)
                self._ready.append(pm)
                # one worker per queued beat (an idle worker that has not woken yet counts once)
                if len(self._ready) > self._idle and self._workers < self.MAX_WORKERS:
                    self._workers += 1
                    threading.Thread(target=self._work, name="mopt-heartbeat-worker",
                                     daemon=True).start()
                self._cv.notify_all()

    def _work(self):
        while True:
            with self._cv:
                self._idle += 1
                deadline = time.monotonic() + self.IDLE_EXIT_S
                while not self._ready:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        self._idle -= 1
                        self._workers -= 1
                        return
                    self._cv.wait(left)
                self._idle -= 1
                pm = self._ready.popleft()
            alive = False
            if not pm.stopped.is_set():
                try:
                    alive = pm._beat()
                except Exception as exc:   # a storage error ends this trial's heartbeat only
                    log.warning("heartbeat of trial %s failed: %s", pm.trial.id, exc)
            with self._cv:
                self._running.discard(pm)
                if alive and not pm.stopped.is_set():
                    self._push(pm, time.monotonic() + pm.wait_time)
                else:
                    pm.stopped.set()
                    self._cv.notify_all()


_SCHEDULER = _Scheduler()


class TrialPacemaker:
    """Keep ``trial``'s heartbeat fresh every ``wait_time`` seconds until it stops running."""

    def __init__(self, trial, wait_time=60, storage=None):
        if storage is None:
            from ..storage.protocol import get_storage
            storage = get_storage()
        self.trial = trial
        self.wait_time = float(wait_time)
        self.storage = storage
        self.stopped = threading.Event()
        self._started = False

    def start(self):
        if self._started:
            raise RuntimeError("a pacemaker starts once")
        self._started = True
        _SCHEDULER.add(self, time.monotonic() + self.wait_time)

    def stop(self):
        """Cancel further beats; returns once none of this trial's beats is in progress."""
        self.stopped.set()
        _SCHEDULER.wait_idle(self)

    def is_alive(self) -> bool:
        return self._started and not self.stopped.is_set()

    def _beat(self) -> bool:
        """One refresh; False when the trial no longer runs here."""
        current = self.storage.get_trial(self.trial)
        if current is None or current.status in STOPPED_STATUS:
            return False
        return bool(self.storage.update_heartbeat(current))
