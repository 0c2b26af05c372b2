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
import ctypes
import logging
import mmap
import multiprocessing as mp
import os
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

    def _take(self, limit: int = 256):
        """Next unit of work: up to ``limit`` queued writes, in order."""
        held = self._held
        n = min(limit, len(held))
        return [held.popleft() for _ in range(n)]

    def _apply_batch(self, held):
        """Apply a unit: one bulk insert of its registrations and one bulk compare-and-swap of
        its updates.  An update of a trial registered in the same unit (a result that arrived
        while the registration still waited, the usual case in a lagging writer child) is merged
        into the document before it is inserted -- one write instead of two.  The updates of
        trials registered earlier go first: an update queued before its trial's registration
        must not see the document (it would not have, applied in order).  A registration that
        hits the unique index (a replay after a writer failover) is skipped and the updates
        merged into it are applied to the stored document instead, as they would have been."""
        b = self.builder
        docs: dict = {}
        merged: dict = {}
        updates = []
        for kind, x in held:
            if kind == "register":
                d = x if type(x) is dict else b.doc(x)
                if d["_id"] not in docs:
                    docs[d["_id"]] = d
                continue
            uid, f, was = x
            if type(f) is not dict:
                f = b.result_fields(f)
            d = docs.get(uid)
            if d is None:
                updates.append((uid, f, was))
                continue
            merged.setdefault(uid, []).append((f, was))
            if was is None or d.get("status") == was:
                d.update(f)
        if updates:
            # the sweep's literals / result_fields are built for this write: the storage may
            # keep them as they are
            self._call("update_trial_docs", updates, owned=True)
        if not docs:
            return
        if self._call("register_trial_docs", list(docs.values()), owned=True):
            return
        for uid, d in docs.items():   # a bulk insert hit a duplicate: insert one by one
            if not self._call("register_trial_docs", [dict(d)]) and uid in merged:
                self._call("update_trial_docs", [(uid, f, was) for f, was in merged[uid]])

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

    def drain_all(self, unit: int) -> None:
        """Apply every held write in units of up to ``unit`` (the writer child's backlog)."""
        t0 = time.perf_counter()
        while self._held:
            with self._lock:
                if self._held:
                    self._apply_batch(self._take(unit))
        self.busy_s += time.perf_counter() - t0

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
    import gc
    gc.set_threshold(20000, 10, 10)   # as the sweep's rank 0 (PopulationSweep.__init__)
    storage = _open(spec)
    if seed_docs:
        storage.database.write("trials", seed_docs)
    wb = WriteBehind(storage, builder)
    while True:
        try:
            msg = conn.recv()
        except EOFError:                    # the parent is gone
            wb.flush()
            return
        if msg[0] == "ops":
            # everything already waiting is applied as one backlog: a lagging child merges a
            # trial's registration and its result into one insert (WriteBehind._apply_batch)
            n = 0
            gone = False
            while msg is not None and msg[0] == "ops":
                n += len(msg[1])
                wb.extend(msg[1])
                try:
                    msg = conn.recv() if conn.poll() else None
                except EOFError:            # the parent died mid-backlog: apply what arrived
                    msg, gone = None, True
            wb.drain_all(4096)
            if gone:
                wb.flush()
                return
            if applied is not None:         # the parent's view of the child's backlog
                applied.value += n
            gc.freeze()                     # the applied documents live on: out of the GC scan
            if msg is None:
                continue
        kind = msg[0]
        wb.flush()
        if kind == "flush":
            conn.send(("flushed", wb.errors))
        elif kind == "dump":           # pickled straight from the child's store (no copies)
            db = storage.database
            read = getattr(db, "read_owned", db.read)
            conn.send(("docs", read("trials", {"experiment": builder.exp_id})))
        elif kind == "close":
            conn.send(("closed", wb.errors))
            return


def _child_main(fd: int, counter_fd: int):  # pragma: no cover - child process
    """Entry point of the writer child (``python -c``, see :class:`_Child`): the arguments
    arrive as the first message; ``counter_fd`` is an 8-byte shared mapping that publishes the
    number of applied writes."""
    import ctypes
    import mmap
    from multiprocessing.connection import Connection
    conn = Connection(fd)
    buf = mmap.mmap(counter_fd, 8)
    spec, builder, seed_docs = conn.recv()
    _child(conn, spec, builder, seed_docs, ctypes.c_int64.from_buffer(buf))


class _Child:
    """The writer child as a plain ``python -c`` subprocess rather than a ``multiprocessing``
    spawn: a spawned child re-imports the parent's ``__main__`` (the sweep, bench.py: torch and
    the whole package, ~2 s and ~300 MB) before it reads its first message, and the sweep's
    first writes -- the initial fill of every slot -- waited that long in the pipe.  This child
    imports the storage layer only."""

    def __init__(self, conn_fd: int, counter_fd: int):
        import os
        import subprocess
        import sys
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"]
                                    if env.get("PYTHONPATH") else "")
        code = ("import sys; from metaopt_amd.worker.writer import _child_main; "
                "_child_main(int(sys.argv[1]), int(sys.argv[2]))")
        self._p = subprocess.Popen([sys.executable, "-c", code, str(conn_fd), str(counter_fd)],
                                   pass_fds=(conn_fd, counter_fd), env=env)

    def is_alive(self) -> bool:
        return self._p.poll() is None

    @property
    def exitcode(self):
        return self._p.poll()

    def kill(self) -> None:
        if self._p.poll() is None:
            self._p.kill()

    def join(self, timeout=None) -> None:
        import subprocess
        try:
            self._p.wait(timeout)
        except subprocess.TimeoutExpired:
            pass


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
        self._conn, child = mp.Pipe()
        # ops applied by the child (a shared 8-byte mapping, no pipe traffic): len(writer)
        # counts the child's backlog too, so the sweep's backlog bound also holds when it lags
        counter_fd = os.memfd_create("mopt-writer-applied")
        os.ftruncate(counter_fd, 8)
        self._counter_map = mmap.mmap(counter_fd, 8)
        self._applied = ctypes.c_int64.from_buffer(self._counter_map)
        self._handed = 0
        self._proc = _Child(child.fileno(), counter_fd)
        child.close()
        os.close(counter_fd)
        self._queue: "queue.SimpleQueue" = queue.SimpleQueue()
        self._queue.put(("init", (spec, builder, seed)))     # the child's first message
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
                if item[0] == "init":
                    self._conn.send(item[1])
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
                if docs:          # unpickled for this call: nobody else holds them
                    if hasattr(db, "insert_owned"):
                        db.insert_owned("trials", docs)
                    else:
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
