"""Storage writes of a device sweep, taken off rank 0's decision path.

A population sweep registers, completes and re-stamps thousands of trials per second; rank 0's
decisions never read those writes back (it keeps its own bookkeeping), so they are queued as
compact specs and applied later:

* :class:`WriteBehind` applies them in the same process, in bulk units, while the GPU still has
  queued work (``drain_while(busy)``) -- enough when rank 0's host has idle time (one GPU);
* :class:`WriterProcess` ships them to a child process that owns its own connection to the
  experiment's database and applies them there -- rank 0's host at 8 GPUs decides for 2,048
  slots per sync and has no idle time left to write in.  An in-memory :class:`EphemeralDB`
  is mirrored: the child starts from a copy of the experiment's trials and the final state is
  copied back at ``close``; file and MongoDB backends are simply opened again in the child.

Both build documents from specs with one :class:`DocBuilder` (the Trial schema of
``core/trial.py``), so a registration costs the decision path one tuple.
"""
from __future__ import annotations

import collections
import logging
import multiprocessing as mp
import threading
import time
from typing import Optional

from ..storage.database import DuplicateKeyError, EphemeralDB, MongoDB, PickledDB

log = logging.getLogger(__name__)


class DocBuilder:
    """Trial documents / result fields of the specs queued by the sweep (picklable)."""

    def __init__(self, exp_id, dim_names, dim_types, sec_name="val_acc"):
        self.exp_id = exp_id
        self.dim_names = list(dim_names)
        self.dim_types = list(dim_types)
        self.sec_name = sec_name

    def doc(self, spec) -> dict:
        tid, stamp, point, parent = spec
        return {"experiment": self.exp_id, "status": "reserved", "worker": None,
                "heartbeat": stamp, "submit_time": stamp, "start_time": stamp,
                "end_time": None, "results": [],
                "params": [{"name": n, "type": t, "value": v}
                           for n, t, v in zip(self.dim_names, self.dim_types, point)],
                "parents": [parent] if parent is not None else [],
                "_id": tid}

    def result_fields(self, spec) -> dict:
        vl, va, tl, now, hb = spec
        return {"results": [{"name": "val_loss", "type": "objective", "value": vl},
                            {"name": self.sec_name, "type": "statistic", "value": va},
                            {"name": "train_loss", "type": "statistic", "value": tl}],
                "status": "completed", "end_time": now, "heartbeat": hb}


class WriteBehind:
    """In-process write-behind queue.

    ``put_*`` queue operations; ``drain_while(busy)`` applies held writes in order, one bulk
    unit at a time, for as long as ``busy()`` says the GPU is still working on queued work (no
    helper thread: it would need the GIL the waiting thread holds).  Consecutive registrations
    become one bulk insert, consecutive updates one bulk compare-and-swap.  ``flush`` applies
    everything.  A lock serialises units so the watchdog thread may flush concurrently.
    """

    def __init__(self, storage, builder: Optional[DocBuilder] = None):
        self.storage = storage
        self.builder = builder
        self.errors = 0
        self._held: "collections.deque" = collections.deque()
        self.busy_s = 0.0             # seconds spent applying writes
        self._lock = threading.Lock()

    # -- queueing ---------------------------------------------------------------------------------
    def put_register(self, doc: dict):
        """Register a trial document (a shallow copy: the sweep replaces, never mutates, the
        fields it changes later)."""
        self._held.append(("register", dict(doc)))

    def put_update(self, uid, fields: dict, was=None):
        """Set ``fields`` of trial ``uid`` (only while its status is ``was``, when given)."""
        self._held.append(("update", (uid, fields, was)))

    def put_register_spec(self, spec: tuple):
        """Register the trial document ``builder.doc(spec)`` (built when the write is applied)."""
        self._held.append(("register", spec))

    def put_update_spec(self, uid, spec: tuple, was=None):
        """Set the fields ``builder.result_fields(spec)`` of trial ``uid`` (built when applied)."""
        self._held.append(("update", (uid, spec, was)))

    def extend(self, items) -> None:
        self._held.extend(items)

    def __len__(self):
        return len(self._held)

    # -- applying ---------------------------------------------------------------------------------
    def drain_while(self, busy) -> None:
        t0 = time.perf_counter()
        while self._held and busy():
            with self._lock:
                if not self._held:
                    break
                self._apply_batch(self._take())
        self.busy_s += time.perf_counter() - t0

    def _take(self):
        """Next unit of work: a run of <= 256 registrations (one bulk insert) or of updates
        (one bulk compare-and-swap)."""
        first = self._held.popleft()
        item = [first]
        while self._held and len(item) < 256 and self._held[0][0] == first[0]:
            item.append(self._held.popleft())
        return item

    def _apply_batch(self, held):
        if held[0][0] == "register":
            docs = [h[1] if type(h[1]) is dict else self.builder.doc(h[1]) for h in held]
            if not self._call("register_trial_docs", docs, owned=True):
                for d in docs:            # a bulk insert hit a duplicate: insert one by one
                    self._call("register_trial_docs", [dict(d)])
            return
        fields = self.builder.result_fields if self.builder is not None else None
        # every queued update carries dicts built for it (the sweep's literals, result_fields):
        # the storage may keep them as they are
        self._call("update_trial_docs",
                   [h[1] if type(h[1][1]) is dict else (h[1][0], fields(h[1][1]), h[1][2])
                    for h in held], owned=True)

    def _call(self, method, *args, **kwargs) -> bool:
        try:
            getattr(self.storage, method)(*args, **kwargs)
            return True
        except DuplicateKeyError:
            log.debug("duplicate write skipped (%s)", method)
            return False
        except Exception as exc:  # pragma: no cover - storage hiccup
            self.errors += 1
            log.warning("storage write %s failed: %s", method, exc)
            return True

    def flush(self):
        """Apply every held write."""
        self.drain_while(lambda: True)

    def close(self):
        self.flush()


# ---------------------------------------------------------------------------------- process
def storage_spec(storage) -> Optional[tuple]:
    """How a child process re-opens ``storage``'s database, or None when it cannot."""
    db = getattr(storage, "database", None)
    if type(db) is EphemeralDB:
        return ("ephemeral",)
    if type(db) is PickledDB:
        return ("pickleddb", db.host)
    if type(db) is MongoDB:
        return ("mongodb", {"host": db.host, "name": db.name, "port": db.port,
                            "username": db.username, "password": db.password})
    return None


def _open(spec):
    from ..storage.protocol import DocumentStorage
    kind = spec[0]
    if kind == "ephemeral":
        return DocumentStorage(EphemeralDB())
    if kind == "pickleddb":
        return DocumentStorage(PickledDB(host=spec[1]))
    return DocumentStorage(MongoDB(**spec[1]))


def _child(conn, spec, builder, seed_docs, applied=None):  # pragma: no cover - child process
    storage = _open(spec)
    if seed_docs:
        storage.database.write("trials", seed_docs)
    wb = WriteBehind(storage, builder)
    while True:
        msg = conn.recv()
        kind = msg[0]
        if kind == "ops":
            wb.extend(msg[1])
            wb.flush()
            if applied is not None:         # the parent's view of the child's backlog
                applied.value += len(msg[1])
        elif kind == "flush":
            wb.flush()
            conn.send(("flushed", wb.errors))
        elif kind == "dump":
            wb.flush()
            conn.send(("docs", storage.database.read("trials", {"experiment": builder.exp_id})))
        elif kind == "close":
            wb.flush()
            conn.send(("closed", wb.errors))
            return


class WriterDied(RuntimeError):
    """The writer child process is gone (it failed to open the database, was killed, or its
    pipe broke)."""


class WriterProcess:
    """:class:`WriteBehind`'s interface, applied by a child process (see module docstring).

    ``drain_while`` only hands the queued specs to a sender thread (pickling and the pipe write
    happen there, while the sweep's thread waits on the GPU or decides), so a slow database
    never blocks the decision path; ``flush``/``close`` wait for the child.

    Failure: when the child dies (or the pipe breaks) the writer falls back to an in-process
    :class:`WriteBehind` on the parent's storage and replays every write the child had not
    acknowledged -- all of them for an in-memory database, whose child copy died with it.  The
    replay is safe: registrations of trials the child did write hit the unique index and are
    skipped, and status updates are compare-and-swap.  No caller ever waits on a dead child:
    requests poll the child's liveness (``poll_s``)."""

    def __init__(self, storage, builder: DocBuilder, spec: tuple, poll_s: float = 0.5):
        import queue
        self.storage = storage
        self.builder = builder
        self.spec = spec
        self.errors = 0
        self.busy_s = 0.0
        self.poll_s = float(poll_s)
        self._held: list = []
        self._lock = threading.Lock()
        # writes handed to the child and not yet covered by an acknowledged flush (an in-memory
        # database keeps them all: the child's copy is the only one until close)
        self._unacked: list = []
        self._failure: Optional[BaseException] = None
        self._fallback: Optional[WriteBehind] = None
        seed = None
        if spec[0] == "ephemeral":
            seed = storage.database.read("trials", {"experiment": builder.exp_id})
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        # ops applied by the child (shared counter, no pipe traffic): len(writer) counts the
        # child's backlog too, so the sweep's backlog bound also holds when the child lags
        self._applied = ctx.Value("q", 0, lock=False)
        self._handed = 0
        self._proc = ctx.Process(target=_child, args=(child, spec, builder, seed, self._applied),
                                 name="mopt-writer", daemon=True)
        self._proc.start()
        child.close()
        self._queue: "queue.SimpleQueue" = queue.SimpleQueue()
        self._sender = threading.Thread(target=self._send_loop, name="mopt-writer-send",
                                        daemon=True)
        self._sender.start()

    put_register = WriteBehind.put_register
    put_update = WriteBehind.put_update
    put_register_spec = WriteBehind.put_register_spec
    put_update_spec = WriteBehind.put_update_spec

    def __len__(self):
        lag = 0 if self._fallback is not None else max(0, self._handed - self._applied.value)
        return len(self._held) + lag

    @property
    def failed(self) -> bool:
        return self._fallback is not None

    def _send_loop(self):
        item = None
        try:
            while True:
                item = self._queue.get()
                if item[0] == "ops":
                    self._conn.send(item)
                    continue
                # ("sync", request, done event, reply box): a request that waits for the child
                _, request, done, box = item
                self._conn.send(request)
                box.append(self._conn.recv())
                done.set()
                item = None
                if request[0] == "close":
                    return
        except BaseException as exc:  # child gone, pipe broken, unpicklable op
            self._failure = exc
            if item is not None and item[0] == "sync":
                item[2].set()           # the waiter sees an empty reply box
            while True:                 # and so does every request queued behind it
                try:
                    nxt = self._queue.get_nowait()
                except Exception:
                    break
                if nxt[0] == "sync":
                    nxt[2].set()

    def _fail_over(self, why) -> WriteBehind:
        """Switch to in-process writes and replay what the child did not acknowledge."""
        if self._fallback is None:
            log.warning("storage writer process failed (%s): writing in process", why)
            fb = WriteBehind(self.storage, self.builder)
            fb.extend(self._unacked)
            self._unacked = []
            self._fallback = fb
            if self._proc is not None and self._proc.is_alive():
                self._proc.kill()
        return self._fallback

    def _hand_over(self):
        with self._lock:
            held, self._held = self._held, []
        if not held:
            return
        if self._fallback is not None:
            self._fallback.extend(held)
            return
        self._unacked.extend(held)
        self._handed += len(held)
        self._queue.put(("ops", held))

    def _request(self, request):
        """Send ``request`` and wait for the reply; None when the child died meanwhile."""
        if self._fallback is not None:
            return None
        done, box = threading.Event(), []
        self._queue.put(("sync", request, done, box))
        while not done.wait(self.poll_s):
            if self._failure is not None or not self._proc.is_alive():
                break
        if box:
            return box[0]
        self._fail_over(self._failure or f"child exited ({self._proc.exitcode})")
        return None

    def drain_while(self, busy) -> None:
        t0 = time.perf_counter()
        if self._fallback is None and (self._failure is not None or not self._proc.is_alive()):
            self._fail_over(self._failure or f"child exited ({self._proc.exitcode})")
        self._hand_over()
        if self._fallback is not None:
            self._fallback.drain_while(busy)
        self.busy_s += time.perf_counter() - t0

    def flush(self):
        """Wait until the child (or the in-process fallback) applied every write so far."""
        self._hand_over()
        reply = self._request(("flush",))
        if reply is not None:
            _, self.errors = reply
            if self.spec[0] != "ephemeral":
                self._unacked = []
            return
        fb = self._fallback
        fb.flush()
        self.errors = fb.errors

    def close(self):
        """Apply everything; copy an in-memory database's trials back into ``storage``."""
        if self._proc is None:
            return
        self._hand_over()
        if self._fallback is None and self.spec[0] == "ephemeral":
            reply = self._request(("dump",))
            if reply is not None:
                _, docs = reply
                db = self.storage.database
                db.remove("trials", {"experiment": self.builder.exp_id})
                if docs:
                    db.write("trials", docs)
                self._unacked = []
        reply = self._request(("close",))
        if reply is not None:
            _, self.errors = reply
        else:
            self._fallback.flush()
            self.errors = self._fallback.errors
        self._proc.join(timeout=60)
        if self._proc.is_alive():
            self._proc.kill()
        self._proc = None
