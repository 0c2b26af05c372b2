"""JSONL event log of a sweep (observability, SURVEY.md §5 "Metrics / logging").

The reference has no event stream: its only run-time record is the trial documents' timestamps
and ``experiment.stats`` (reference src/orion/core/worker/experiment.py:419-467) plus the
end-of-run RESULTS dump (src/orion/core/worker/__init__.py:70-88).  A population sweep completes
thousands of trials per second, so this log is record-oriented and cheap: one JSON object per
line, appended through a buffered file handle, flushed every ``flush_every`` records and at
``close``.

Record schema (every record has ``ts`` -- unix seconds -- and ``event``):

* ``sweep_start``: ``world_size``, ``population``, ``sync_every``, ``algorithm``;
* ``sync``: ``step``, ``completed``, ``broken``, ``active``, ``best`` and the per-phase host
  timers of the interval (``ms``: suggest/observe/collective/apply ...);
* ``trial``: ``id``, ``status`` (completed / broken), ``objective``, ``budget``;
* ``watchdog``: ``stalled_s`` and ``phase`` when the rank-failure watchdog fires;
* ``sweep_end``: the sweep summary.

``read_events(path)`` parses a log back (tests, post-mortems).
"""
from __future__ import annotations

import json
import math
import os
import threading
import time
from typing import IO, Iterator, Optional


def _clean(v):
    """JSON-safe scalars: numpy scalars -> python, non-finite floats -> None."""
    if hasattr(v, "item") and not isinstance(v, (list, dict, str)):
        try:
            v = v.item()
        except (ValueError, AttributeError):
            pass
    if isinstance(v, float) and not math.isfinite(v):
        return None
    if isinstance(v, dict):
        return {str(k): _clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_clean(x) for x in v]
    return v


class EventLog:
    """Append-only JSONL writer, safe to call from the sweep thread and the watchdog thread."""

    def __init__(self, path: str, flush_every: int = 64, rank: int = 0):
        self.path = path
        self.rank = rank
        self.flush_every = max(1, int(flush_every))
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._fh: Optional[IO[str]] = open(path, "a", buffering=1 << 16)
        self._pending = 0
        self._lock = threading.Lock()

    def emit(self, event: str, **fields) -> None:
        rec = {"ts": round(time.time(), 6), "event": event, "rank": self.rank}
        rec.update(_clean(fields))
        line = json.dumps(rec, separators=(",", ":"), default=str)
        with self._lock:
            if self._fh is None:
                return
            self._fh.write(line + "\n")
            self._pending += 1
            if self._pending >= self.flush_every:
                self._fh.flush()
                self._pending = 0

    def flush(self) -> None:
        with self._lock:
            if self._fh is not None:
                self._fh.flush()
                self._pending = 0

    def close(self) -> None:
        with self._lock:
            if self._fh is not None:
                self._fh.flush()
                self._fh.close()
                self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class NullEventLog:
    """Stand-in when no log is requested: every call is a no-op."""

    def emit(self, event: str, **fields) -> None:
        pass

    def flush(self) -> None:
        pass

    def close(self) -> None:
        pass


def read_events(path: str, event: Optional[str] = None) -> Iterator[dict]:
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            rec = json.loads(line)
            if event is None or rec.get("event") == event:
                yield rec
