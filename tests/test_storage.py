"""Database backends and the storage protocol (reference tests: tests/unittests/core/
test_ephemeraldb.py, test_pickleddb.py, tests/unittests/storage/test_storage.py)."""
import datetime
import multiprocessing
import os

import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.storage.database import (DuplicateKeyError, EphemeralDB, PickledDB,
                                          create_database)
from metaopt_amd.storage.protocol import DocumentStorage, FailedUpdate


@pytest.fixture(params=["ephemeral", "pickled", "mongodb"])
def db(request, tmp_path, monkeypatch):
    if request.param == "ephemeral":
        return EphemeralDB()
    if request.param == "mongodb":       # the same contract through a stand-in pymongo
        import fake_pymongo
        fake_pymongo.install(monkeypatch)
        from metaopt_amd.storage.database import MongoDB
        return MongoDB(host="mongodb://user:pass@localhost/mopt_test")
    return PickledDB(host=str(tmp_path / "db.pkl"))


def _fill(db):
    db.write("exps", [{"name": "a", "version": 1, "meta": {"user": "u1", "n": 3}},
                      {"name": "b", "version": 1, "meta": {"user": "u2", "n": 5}},
                      {"name": "a", "version": 2, "meta": {"user": "u1", "n": 7}}])


class TestDatabase:
    def test_insert_assigns_ids_and_reads(self, db):
        doc = {"name": "x"}
        assert db.write("c", doc) == 1
        assert "_id" in doc
        assert db.read("c", {"_id": doc["_id"]})[0]["name"] == "x"

    def test_queries(self, db):
        _fill(db)
        assert len(db.read("exps", {"name": "a"})) == 2
        assert len(db.read("exps", {"meta.user": "u1"})) == 2
        assert len(db.read("exps", {"meta.n": {"$gte": 5}})) == 2
        assert len(db.read("exps", {"meta.n": {"$gt": 5}})) == 1
        assert len(db.read("exps", {"meta.n": {"$lte": 5}})) == 2
        assert len(db.read("exps", {"name": {"$in": ["a", "z"]}})) == 2
        assert len(db.read("exps", {"name": {"$ne": "a"}})) == 1
        assert len(db.read("exps", {"name": {"$nin": ["a"]}})) == 1
        assert len(db.read("exps", {"meta": {"user": "u2"}})) == 1
        assert db.count("exps", {"name": "a"}) == 2
        assert db.count("exps") == 3

    def test_projection(self, db):
        _fill(db)
        docs = db.read("exps", {"name": "b"}, {"meta.user": 1})
        assert docs[0] == {"_id": docs[0]["_id"], "meta": {"user": "u2"}}
        docs = db.read("exps", {"name": "b"}, {"meta": 0, "_id": 0})
        assert docs[0] == {"name": "b", "version": 1}
        with pytest.raises(ValueError):
            db.read("exps", {}, {"name": 1, "version": 0})

    def test_update_and_read_and_write(self, db):
        _fill(db)
        assert db.write("exps", {"meta.n": 0}, {"name": "a"}) == 2
        assert all(d["meta"]["n"] == 0 and d["meta"]["user"] == "u1"
                   for d in db.read("exps", {"name": "a"}))
        doc = db.read_and_write("exps", {"name": "b"}, {"status": "taken"})
        assert doc["status"] == "taken"
        assert db.read_and_write("exps", {"name": "zzz"}, {"x": 1}) is None

    def test_unique_index(self, db):
        db.ensure_index("exps", [("name", EphemeralDB.ASCENDING),
                                 ("version", EphemeralDB.ASCENDING)], unique=True)
        _fill(db)
        assert db.index_information("exps")["name_1_version_1"] is True
        with pytest.raises(DuplicateKeyError):
            db.write("exps", {"name": "a", "version": 2})
        with pytest.raises(DuplicateKeyError):
            db.write("exps", {"version": 2}, {"name": "a", "version": 1})
        db.drop_index("exps", "name_1_version_1")
        db.write("exps", {"name": "a", "version": 2})

    def test_remove(self, db):
        _fill(db)
        assert db.remove("exps", {"name": "a"}) == 2
        assert db.count("exps") == 1

    def test_duplicate_id(self, db):
        db.write("c", {"_id": "k", "v": 1})
        with pytest.raises(DuplicateKeyError):
            db.write("c", {"_id": "k", "v": 2})


def _concurrent_writer(args):
    path, i = args
    db = PickledDB(host=path)
    try:
        db.write("concurrent", {"_id": i % 5, "writer": i})
        return 1
    except DuplicateKeyError:
        return 0


def test_pickleddb_concurrent_unique_writes(tmp_path):
    """10 processes race to insert 5 unique ids: exactly 5 succeed (reference
    test_pickleddb.py:335-356)."""
    path = str(tmp_path / "race.pkl")
    PickledDB(host=path).ensure_index("concurrent", "_id", unique=True)
    ctx = multiprocessing.get_context("spawn")
    with ctx.Pool(4) as pool:
        res = pool.map(_concurrent_writer, [(path, i) for i in range(10)])
    assert sum(res) == 5
    assert PickledDB(host=path).count("concurrent") == 5


def test_create_database_by_name(tmp_path):
    assert isinstance(create_database("EphemeralDB"), EphemeralDB)
    assert isinstance(create_database("pickleddb", host=str(tmp_path / "x.pkl")), PickledDB)


class _Exp:
    def __init__(self, _id):
        self._id = _id


@pytest.fixture(params=["ephemeral", "mongodb"])
def storage(request, monkeypatch):
    if request.param == "mongodb":
        import fake_pymongo
        fake_pymongo.install(monkeypatch)
        from metaopt_amd.storage.database import MongoDB
        return DocumentStorage(MongoDB(host="mongodb://user:pass@localhost/mopt_test"),
                               heartbeat=120)
    return DocumentStorage(EphemeralDB(), heartbeat=120)


def _trial(exp, x, status="new"):
    t = Trial(experiment=exp._id, status=status, params=[dict(name="/x", type="real", value=x)])
    t.submit_time = datetime.datetime.utcnow()
    return t


class TestStorageProtocol:
    def test_experiment_unique_name_version(self, storage):
        storage.create_experiment({"name": "e", "version": 1, "metadata": {}})
        with pytest.raises(DuplicateKeyError):
            storage.create_experiment({"name": "e", "version": 1, "metadata": {}})

    def test_register_dedup(self, storage):
        exp = _Exp("E")
        storage.register_trial(_trial(exp, 1.0))
        with pytest.raises(DuplicateKeyError):
            storage.register_trial(_trial(exp, 1.0))

    def test_reserve_is_exclusive(self, storage):
        exp = _Exp("E")
        for x in range(3):
            storage.register_trial(_trial(exp, float(x)))
        got = [storage.reserve_trial(exp) for _ in range(4)]
        assert sum(t is not None for t in got) == 3
        assert len({t.id for t in got if t}) == 3
        assert all(t.status == "reserved" and t.heartbeat is not None for t in got if t)

    def test_cas_status(self, storage):
        exp = _Exp("E")
        storage.register_trial(_trial(exp, 1.0))
        t = storage.reserve_trial(exp)
        stale = Trial(**t.to_dict())
        storage.set_trial_status(t, "interrupted")
        with pytest.raises(FailedUpdate):
            storage.set_trial_status(stale, "completed")
        assert storage.get_trial(t).status == "interrupted"

    def test_lost_trials(self, storage):
        exp = _Exp("E")
        storage.register_trial(_trial(exp, 1.0))
        t = storage.reserve_trial(exp)
        assert storage.fetch_lost_trials(exp) == []
        old = datetime.datetime.utcnow() - datetime.timedelta(seconds=1000)
        storage._db.write("trials", {"heartbeat": old}, {"_id": t.id})
        assert [x.id for x in storage.fetch_lost_trials(exp)] == [t.id]

    def test_results_file(self, storage, tmp_path):
        exp = _Exp("E")
        storage.register_trial(_trial(exp, 1.0))
        t = storage.reserve_trial(exp)
        f = tmp_path / "results.json"
        f.write_text('[{"name": "loss", "type": "objective", "value": 0.5}]')
        storage.retrieve_result(t, str(f))
        t.status = "completed"
        storage.push_trial_results(t)
        assert storage.count_completed_trials(exp) == 1
        assert storage.get_trial(t).objective.value == 0.5

    def test_counts_and_status_queries(self, storage):
        exp = _Exp("E")
        for i, st in enumerate(["new", "completed", "broken", "broken", "suspended"]):
            storage.register_trial(_trial(exp, float(i), status=st))
        assert storage.count_broken_trials(exp) == 2
        assert storage.count_completed_trials(exp) == 1
        assert len(storage.fetch_pending_trials(exp)) == 2
        assert len(storage.fetch_noncompleted_trials(exp)) == 4
        assert len(storage.fetch_trials_by_status(exp, "broken")) == 2


def test_writer_process_mirrors_ephemeral_db():
    """The sweep's child-process writer applies queued specs in its own copy of an in-memory
    database and copies the final trials back at close; file databases are shared."""
    import datetime
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.writer import DocBuilder, WriterProcess, storage_spec
    storage = DocumentStorage(EphemeralDB())
    storage.database.write("trials", {"_id": "old", "experiment": 7, "status": "interrupted",
                                      "params": [], "results": []})
    b = DocBuilder(7, ["/x"], ["real"])
    w = WriterProcess(storage, b, storage_spec(storage))
    now = datetime.datetime.utcnow()
    for i in range(300):
        w.put_register_spec((f"t{i}", now, (float(i),), None))
    w.put_update("old", {"status": "reserved"}, was="interrupted")
    w.drain_while(lambda: True)
    w.put_update_spec("t3", (0.5, 0.9, 0.7, now, now), was="reserved")
    w.flush()
    w.close()
    docs = {d["_id"]: d for d in storage.database.read("trials", {"experiment": 7})}
    assert len(docs) == 301 and docs["old"]["status"] == "reserved"
    assert docs["t3"]["status"] == "completed" and docs["t3"]["results"][0]["value"] == 0.5
    assert docs["t5"]["params"][0] == {"name": "/x", "type": "real", "value": 5.0}


def test_write_behind_merges_results_into_pending_registrations():
    """A unit holding a trial's registration and its later result inserts ONE completed
    document; the ordering cases keep their applied-in-order meaning: an update queued before
    its trial's registration finds nothing, a compare-and-swap that does not match is dropped,
    and a duplicate registration (failover replay) applies its merged updates to the stored
    document instead."""
    import datetime
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.writer import DocBuilder, WriteBehind
    storage = DocumentStorage(EphemeralDB())
    b = DocBuilder(7, ["/x"], ["real"])
    now = datetime.datetime.utcnow()
    w = WriteBehind(storage, b)
    w.put_register_spec(("dup", now, (0.0,), None))
    w.flush()
    calls = []
    real = storage.update_trial_docs
    storage.update_trial_docs = lambda items, owned=False: (calls.append(len(items)),
                                                           real(items, owned))[1]
    w.put_update("early", {"status": "broken"}, was="reserved")     # before its registration
    for i in range(4):
        w.put_register_spec((f"t{i}", now, (float(i),), None))
    w.put_update_spec("t1", (0.5, 0.9, 0.7, now, now), was="reserved")
    w.put_update("t2", {"status": "broken", "heartbeat": now}, was="reserved")
    w.put_update_spec("t2", (0.1, 0.9, 0.7, now, now), was="reserved")   # CAS fails: broken
    w.put_register_spec(("early", now, (9.0,), None))
    w.flush()
    # the merged results cost no update: one bulk update, for the trial registered earlier
    assert calls == [1]
    w.put_register_spec(("dup", now, (0.0,), None))                       # already stored
    w.put_update_spec("dup", (0.3, 0.9, 0.7, now, now), was="reserved")
    w.flush()
    docs = {d["_id"]: d for d in storage.database.read("trials", {"experiment": 7})}
    assert len(docs) == 6
    assert docs["t1"]["status"] == "completed" and docs["t1"]["results"][0]["value"] == 0.5
    assert docs["t2"]["status"] == "broken" and docs["t2"]["results"] == []
    assert docs["t0"]["status"] == docs["early"]["status"] == "reserved"
    assert docs["dup"]["status"] == "completed" and docs["dup"]["results"][0]["value"] == 0.3


def test_writer_process_killed_child_falls_back_in_process():
    """A writer child that dies (OOM kill, crash) never hangs flush/close: the writer notices,
    switches to in-process writes and replays what the child had not acknowledged -- for an
    in-memory database, every write (the child's copy died with it)."""
    import datetime
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.writer import DocBuilder, WriterProcess, storage_spec
    storage = DocumentStorage(EphemeralDB())
    b = DocBuilder(7, ["/x"], ["real"])
    w = WriterProcess(storage, b, storage_spec(storage), poll_s=0.1)
    now = datetime.datetime.utcnow()
    for i in range(20):
        w.put_register_spec((f"t{i}", now, (float(i),), None))
    w.flush()
    w._proc.kill()
    w._proc.join(timeout=10)
    for i in range(20, 30):
        w.put_register_spec((f"t{i}", now, (float(i),), None))
    w.put_update_spec("t3", (0.5, 0.9, 0.7, now, now), was="reserved")
    w.flush()                       # returns: the child is gone
    assert w.failed
    w.put_register_spec(("late", now, (99.0,), None))
    w.close()
    docs = {d["_id"]: d for d in storage.database.read("trials", {"experiment": 7})}
    assert len(docs) == 31 and docs["t3"]["status"] == "completed"
    assert docs["late"]["params"][0]["value"] == 99.0


def test_writer_child_applies_backlog_when_parent_dies_mid_drain(tmp_path):
    """the child's backlog drain polled then received; a dead parent makes poll()
    true and recv() raise EOFError -- the writes already taken from the pipe must still land."""
    import datetime
    from metaopt_amd.storage.database import PickledDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.writer import DocBuilder, _child
    path = str(tmp_path / "db.pkl")
    b = DocBuilder(7, ["/x"], ["real"])
    now = datetime.datetime.utcnow()
    ops = [("register", (f"t{i}", now, (float(i),), None)) for i in range(6)]

    class DeadParentConn:
        def __init__(self, msgs):
            self.msgs = list(msgs)

        def recv(self):
            if not self.msgs:
                raise EOFError
            return self.msgs.pop(0)

        def poll(self):
            return True          # a closed pipe polls readable

        def send(self, msg):
            raise AssertionError("nothing is sent to a dead parent")

    _child(DeadParentConn([("ops", ops[:3]), ("ops", ops[3:])]), ("pickleddb", path), b, None)
    docs = DocumentStorage(PickledDB(host=path)).database.read("trials", {"experiment": 7})
    assert sorted(d["_id"] for d in docs) == [f"t{i}" for i in range(6)]


def test_writer_process_child_that_cannot_open_the_database(tmp_path):
    """A child that fails at start-up (here: a PickledDB path whose parent is a file) is seen
    as dead; the writes land through the parent's own storage."""
    import datetime
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.writer import DocBuilder, WriterProcess
    storage = DocumentStorage(EphemeralDB())
    blocker = tmp_path / "file"
    blocker.write_text("x")
    b = DocBuilder(7, ["/x"], ["real"])
    w = WriterProcess(storage, b, ("pickleddb", str(blocker / "sub" / "db.pkl")), poll_s=0.1)
    now = datetime.datetime.utcnow()
    for i in range(5):
        w.put_register_spec((f"t{i}", now, (float(i),), None))
    w.flush()
    w.close()
    assert w.failed
    assert len(storage.database.read("trials", {"experiment": 7})) == 5


def test_mongodb_uri_and_connection_errors(monkeypatch):
    """URI parsing (user, password, database, port) and server errors surfacing as
    DatabaseError (reference: src/orion/core/io/database/mongodb.py:30-86,272-295)."""
    import fake_pymongo
    fake_pymongo.install(monkeypatch)
    from metaopt_amd.storage.database import DatabaseError, MongoDB
    db = MongoDB(host="mongodb://alice:s3cret@localhost:27018/studies")
    assert (db.username, db.password, db.name, db.port) == ("alice", "s3cret", "studies", 27018)
    with pytest.raises(DatabaseError):
        MongoDB(host="mongodb://unreachable:1/x")
    with pytest.raises(DatabaseError):
        db.drop_index("trials", "no_such_index")


def test_pickleddb_older_format_is_upgraded(tmp_path, monkeypatch, capsys):
    """A PickledDB file in the first release's layout (indexes keyed by their field tuple, no
    hash indexes) loads, and ``mopt db upgrade`` rewrites it in the current format with the
    deprecated (name, metadata.user) index dropped and the unique indexes still enforced."""
    import pickle
    from metaopt_amd import cli
    from metaopt_amd.storage import database as dbm
    from metaopt_amd.storage import protocol
    path = tmp_path / "old.pkl"
    eph = EphemeralDB()
    eph.write("experiments", {"name": "e", "version": 1,
                              "metadata": {"user": "u", "user_args": ["-x~uniform(0, 1)"]}})
    eph.ensure_index("experiments", [("name", 1), ("metadata.user", 1)], unique=True)

    def legacy_state(col):          # the old layout: field-tuple keys, value sets, no hashes
        return {"docs": col.docs, "_next_id": col._next_id,
                "indexes": {f: (f, u, v) for _, (f, u, v) in col.indexes.items()}}
    monkeypatch.setattr(dbm._Collection, "__getstate__", legacy_state)
    path.write_bytes(pickle.dumps(eph))
    monkeypatch.undo()
    old = PickledDB(host=str(path))
    assert old.read("experiments", {"name": "e"})[0]["version"] == 1
    assert "name_1_metadata.user_1" in old.index_information("experiments")
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(path))
    monkeypatch.setattr(protocol, "_STORAGE", None)
    assert cli.main(["db", "upgrade", "-f"]) == 0
    out = capsys.readouterr().out
    assert "Updating pickleddb scheme" in out
    assert "2 collection(s) converted to format 2" in out or "1 collection(s) converted" in out
    raw = pickle.loads(path.read_bytes())
    assert all(col.__getstate__()["format"] == 2 and not col.migrated
               for col in raw._db.values())
    new = PickledDB(host=str(path))
    assert "name_1_metadata.user_1" not in new.index_information("experiments")
    exp = new.read("experiments", {"name": "e"})[0]
    assert exp["metadata"]["priors"] == {"/x": "uniform(0, 1)"}
    with pytest.raises(DuplicateKeyError):
        new.write("experiments", {"_id": exp["_id"], "name": "other"})
