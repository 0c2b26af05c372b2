"""Storage protocol: experiments, trials and lies on top of a document database.

Behavioural parity with the reference's ``src/orion/storage/base.py:28-281`` and
``src/orion/storage/legacy.py:24-309``:

* indexes: unique ``(name, version)`` on experiments, plus ``metadata.datetime`` and the trial
  indexes ``experiment``, ``status``, ``results``, ``start_time``, ``end_time`` (desc);
* **atomic reserve**: one ``read_and_write`` on ``{experiment, status in [interrupted, new,
  suspended]}`` setting ``status='reserved', start_time, heartbeat``;
* **CAS status updates**: ``where={'_id', 'status': old}``, raising :class:`FailedUpdate` when
  another worker changed the trial first;
* **lost trials**: reserved trials whose heartbeat is older than ``heartbeat`` seconds;
* trial registration dedups through the unique ``_id`` (md5 of the params).

The process-wide storage is set with :func:`setup_storage` and read with :func:`get_storage`
(the reference's ``Storage`` singleton factory).
"""
from __future__ import annotations

import datetime
import json
import logging
from typing import List, Optional

from ..core.trial import Trial
from ..utils.registry import Registry
from .database import (AbstractDB, DatabaseError, EphemeralDB, OutdatedDatabaseError, ReadOnlyDB,
                       create_database)

log = logging.getLogger(__name__)


class FailedUpdate(DatabaseError):
    """A compare-and-swap update matched no document (another worker won the race)."""


class MissingArguments(ValueError):
    pass


def utcnow() -> datetime.datetime:
    return datetime.datetime.utcnow()


def db_is_outdated(db: AbstractDB) -> bool:
    """Deprecated index layout of old databases (reference ``core/utils/backward.py:30-34``)."""
    try:
        info = db.index_information("experiments")
    except Exception:  # pragma: no cover - backend without the collection
        return False
    return "name_1_metadata.user_1" in info


# storage protocols by name (``storage: {type: legacy}``); plugins through the ``Storage`` entry
# point group, as the reference declares its own (reference setup.py:48-50)
STORAGES = Registry("Storage", groups=("metaopt_amd.storages", "Storage"))


class BaseStorageProtocol:
    """Interface every storage backend implements."""

    def create_experiment(self, config):
        raise NotImplementedError

    def update_experiment(self, experiment=None, uid=None, where=None, **kwargs):
        raise NotImplementedError

    def fetch_experiments(self, query, selection=None):
        raise NotImplementedError

    def register_trial(self, trial):
        raise NotImplementedError

    def register_lie(self, trial):
        raise NotImplementedError

    def reserve_trial(self, experiment):
        raise NotImplementedError

    def fetch_trials(self, experiment=None, uid=None):
        raise NotImplementedError

    def get_trial(self, trial=None, uid=None):
        raise NotImplementedError

    def fetch_lost_trials(self, experiment):
        raise NotImplementedError

    def retrieve_result(self, trial, results_file=None, **kwargs):
        raise NotImplementedError

    def push_trial_results(self, trial):
        raise NotImplementedError

    def set_trial_status(self, trial, status, heartbeat=None):
        raise NotImplementedError

    def fetch_pending_trials(self, experiment):
        raise NotImplementedError

    def fetch_noncompleted_trials(self, experiment):
        raise NotImplementedError

    def fetch_trials_by_status(self, experiment, status):
        raise NotImplementedError

    def count_completed_trials(self, experiment):
        raise NotImplementedError

    def count_broken_trials(self, experiment):
        raise NotImplementedError

    def update_heartbeat(self, trial):
        raise NotImplementedError


def _uid(obj, uid, what):
    if obj is not None and uid is not None:
        assert getattr(obj, "_id", getattr(obj, "id", None)) == uid
    if uid is None:
        if obj is None:
            raise MissingArguments(f"Either `{what}` or `uid` should be set")
        uid = getattr(obj, "_id", None) if what == "experiment" else obj.id
    return uid


@STORAGES.register("legacy")
class DocumentStorage(BaseStorageProtocol):
    """The reference's ``Legacy`` protocol: everything in one document database."""

    def __init__(self, database: Optional[AbstractDB] = None, setup: bool = True,
                 heartbeat: float = 120.0):
        self._db = database if database is not None else EphemeralDB()
        self.heartbeat = heartbeat
        if setup:
            self._setup_db()

    @property
    def database(self) -> AbstractDB:
        return self._db

    def _setup_db(self):
        if db_is_outdated(self._db):
            raise OutdatedDatabaseError("The database is outdated. You can upgrade it with the "
                                        "command `mopt db upgrade`.")
        A, D = AbstractDB.ASCENDING, AbstractDB.DESCENDING
        self._db.ensure_index("experiments", [("name", A), ("version", A)], unique=True)
        self._db.ensure_index("experiments", "metadata.datetime")
        self._db.ensure_index("trials", "experiment")
        self._db.ensure_index("trials", "status")
        self._db.ensure_index("trials", "results")
        self._db.ensure_index("trials", "start_time")
        self._db.ensure_index("trials", [("end_time", D)])

    # -- experiments ------------------------------------------------------------------------------
    def create_experiment(self, config):
        return self._db.write("experiments", data=config, query=None)

    def update_experiment(self, experiment=None, uid=None, where=None, **kwargs):
        uid = _uid(experiment, uid, "experiment")
        where = dict(where or {})
        where["_id"] = uid
        return self._db.write("experiments", data=kwargs, query=where)

    def fetch_experiments(self, query, selection=None):
        return self._db.read("experiments", query, selection)

    def delete_experiment(self, experiment=None, uid=None):
        uid = _uid(experiment, uid, "experiment")
        self._db.remove("trials", {"experiment": uid})
        self._db.remove("lying_trials", {"experiment": uid})
        self._db.remove("algo_state", {"experiment": uid})
        return self._db.remove("experiments", {"_id": uid})

    # -- algorithm state ----------------------------------------------------------------------------
    # The reference never persists algorithm state: a worker rebuilds it by replaying every
    # completed trial through ``observe`` (src/orion/core/worker/producer.py:103-132).  A device
    # sweep completes thousands of trials per second, so the algorithm's ``state_dict`` is stored
    # instead (one document per experiment, SURVEY.md §5 "Checkpoint / resume") and restored on
    # re-run with ``set_state``.
    def save_algorithm_state(self, experiment=None, uid=None, state=None) -> None:
        uid = _uid(experiment, uid, "experiment")
        doc = {"state": state, "updated": utcnow()}
        if not self._db.write("algo_state", data=doc, query={"experiment": uid}):
            doc["experiment"] = uid
            self._db.write("algo_state", data=doc)

    def get_algorithm_state(self, experiment=None, uid=None) -> Optional[dict]:
        uid = _uid(experiment, uid, "experiment")
        docs = self._db.read("algo_state", {"experiment": uid})
        return docs[0]["state"] if docs else None

    # -- trials -----------------------------------------------------------------------------------
    def fetch_trials(self, experiment=None, uid=None, query=None):
        uid = _uid(experiment, uid, "experiment")
        q = {"experiment": uid}
        if query:
            q.update(query)
        return self._fetch_trials(q)

    def _fetch_trials(self, query, selection=None) -> List[Trial]:
        trials = Trial.build(self._db.read("trials", query=query, selection=selection))
        trials.sort(key=lambda t: t.submit_time or datetime.datetime.min)
        return trials

    def register_trial(self, trial: Trial) -> Trial:
        self._db.write("trials", trial.to_dict())
        return trial

    def register_trials(self, trials: List[Trial]) -> int:
        """Bulk registration (device populations register hundreds of trials per suggest)."""
        return self._db.write("trials", [t.to_dict() for t in trials])

    def register_trial_docs(self, docs: List[dict], owned: bool = False) -> int:
        """Bulk registration of ready-made trial documents (the Trial schema, ``_id`` included):
        the device sweep builds them without Trial objects.  ``owned``: the caller never touches
        them again, so an in-process backend may keep them without copying."""
        if owned and hasattr(self._db, "insert_owned"):
            return self._db.insert_owned("trials", docs)
        return self._db.write("trials", list(docs))

    def update_trial_doc(self, uid, fields: dict, was: Optional[str] = None) -> int:
        """Set ``fields`` of trial ``uid`` (compare-and-swap on the status when ``was`` is set)."""
        return self.update_trial_docs([(uid, fields, was)])

    def update_trial_docs(self, items, owned: bool = False) -> int:
        """Bulk :meth:`update_trial_doc`: ``items`` = [(uid, fields, was or None)]; ``owned``:
        the caller hands the field values over (an in-process backend keeps them uncopied)."""
        if hasattr(self._db, "set_fields_by_id"):
            return self._db.set_fields_by_id("trials", items, owned=owned)
        n = 0
        for uid, fields, was in items:
            where = {"_id": uid}
            if was is not None:
                where["status"] = was
            n += self._db.write("trials", data=fields, query=where)
        return n

    def register_lie(self, trial: Trial):
        return self._db.write("lying_trials", trial.to_dict())

    def fetch_lies(self, experiment):
        return Trial.build(self._db.read("lying_trials", {"experiment": experiment._id}))

    def retrieve_result(self, trial: Trial, results_file=None, **kwargs) -> Trial:
        """Parse the user script's JSON results file into ``trial.results`` (no DB write)."""
        path = getattr(results_file, "name", results_file)
        with open(path) as f:
            text = f.read()
        results = json.loads(text) if text.strip() else []
        trial.results = [Trial.Result(name=r["name"], type=r["type"], value=r["value"])
                         for r in results]
        return trial

    def get_trial(self, trial=None, uid=None) -> Optional[Trial]:
        uid = _uid(trial, uid, "trial")
        res = self._db.read("trials", {"_id": uid})
        return Trial(**res[0]) if res else None

    def _update_trial(self, trial: Trial, where=None, **kwargs):
        where = dict(where or {})
        where["_id"] = trial.id
        return self._db.write("trials", data=kwargs, query=where)

    def fetch_lost_trials(self, experiment) -> List[Trial]:
        threshold = utcnow() - datetime.timedelta(seconds=self.heartbeat)
        return self._fetch_trials({"experiment": experiment._id, "status": "reserved",
                                   "heartbeat": {"$lte": threshold}})

    def push_trial_results(self, trial: Trial):
        d = trial.to_dict()
        d.pop("_id")
        return self._update_trial(trial, **d)

    def complete_trial(self, trial: Trial) -> int:
        """Write the outcome of a finished trial: results, status, end time and heartbeat only
        (the other fields are unchanged since registration, so the document ends up identical
        to :meth:`push_trial_results` at a fraction of the cost)."""
        return self._update_trial(trial, results=[r.to_dict() for r in trial.results],
                                  status=trial.status, end_time=trial.end_time,
                                  heartbeat=trial.heartbeat)

    def set_trial_status(self, trial: Trial, status: str, heartbeat=None, was=None):
        """CAS: move ``trial`` from its current status (or ``was``) to ``status``."""
        heartbeat = heartbeat or utcnow()
        update = dict(status=status, heartbeat=heartbeat, experiment=trial.experiment)
        old = was if was is not None else trial.status
        if old == "new":
            update["start_time"] = utcnow()
        elif status == "completed":
            update["end_time"] = utcnow()
        rc = self._update_trial(trial, where={"status": old}, **update)
        if not rc:
            raise FailedUpdate(f"trial {trial.id} is no longer '{old}'")
        trial.status = status
        for k in ("start_time", "end_time", "heartbeat"):
            if k in update:
                setattr(trial, k, update[k])

    def fetch_pending_trials(self, experiment):
        return self._fetch_trials({"experiment": experiment._id,
                                   "status": {"$in": ["new", "suspended", "interrupted"]}})

    def reserve_trial(self, experiment) -> Optional[Trial]:
        now = utcnow()
        doc = self._db.read_and_write(
            "trials",
            query={"experiment": experiment._id,
                   "status": {"$in": ["interrupted", "new", "suspended"]}},
            data={"status": "reserved", "start_time": now, "heartbeat": now})
        return Trial(**doc) if doc is not None else None

    def fetch_noncompleted_trials(self, experiment):
        return self._fetch_trials({"experiment": experiment._id, "status": {"$ne": "completed"}})

    def fetch_trials_by_status(self, experiment, status):
        return self._fetch_trials({"experiment": experiment._id, "status": status})

    fetch_trial_by_status = fetch_trials_by_status  # reference spelling

    def count_completed_trials(self, experiment) -> int:
        return self._db.count("trials", {"experiment": experiment._id, "status": "completed"})

    def count_broken_trials(self, experiment) -> int:
        return self._db.count("trials", {"experiment": experiment._id, "status": "broken"})

    def count_trials(self, experiment, status=None) -> int:
        q = {"experiment": experiment._id}
        if status is not None:
            q["status"] = status
        return self._db.count("trials", q)

    def update_heartbeat(self, trial: Trial):
        return self._update_trial(trial, where={"status": "reserved"}, heartbeat=utcnow())


class ReadOnlyStorage:
    """Read-only facade handed to experiment views (reference ``storage/base.py:251-281``)."""

    __slots__ = ("_storage",)
    valid_attributes = {"fetch_trials", "fetch_experiments", "count_broken_trials",
                        "count_completed_trials", "count_trials", "fetch_noncompleted_trials",
                        "fetch_pending_trials", "fetch_lost_trials", "fetch_trials_by_status",
                        "fetch_trial_by_status", "get_trial", "fetch_lies", "database"}

    def __init__(self, storage):
        self._storage = storage

    def __getattr__(self, attr):
        if attr not in self.valid_attributes:
            raise AttributeError(f"Cannot access attribute {attr} on view-only experiments.")
        val = getattr(self._storage, attr)
        if attr == "database":
            return ReadOnlyDB(val)
        return val


_STORAGE: Optional[DocumentStorage] = None


def setup_storage(config: Optional[dict] = None, debug: bool = False,
                  heartbeat: Optional[float] = None) -> DocumentStorage:
    """Create the process-wide storage from ``{'type': 'legacy', 'database': {...}}``."""
    global _STORAGE
    config = dict(config or {})
    db_cfg = dict(config.get("database") or {})
    of_type = db_cfg.pop("type", "pickleddb")
    if debug or config.get("debug"):
        of_type = "ephemeraldb"
    if heartbeat is None:
        from ..core.config import config as global_config
        heartbeat = global_config.worker.heartbeat
    db = create_database(of_type, **db_cfg)
    _STORAGE = STORAGES.get(config.get("type", "legacy"))(db, heartbeat=heartbeat)
    return _STORAGE


def set_storage(storage: Optional[DocumentStorage]) -> None:
    global _STORAGE
    _STORAGE = storage


def get_storage() -> DocumentStorage:
    if _STORAGE is None:
        raise RuntimeError("No storage configured: call setup_storage() first")
    return _STORAGE


def storage_is_set() -> bool:
    return _STORAGE is not None
