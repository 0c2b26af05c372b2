"""Document databases: the control plane shared by every worker of an experiment.

Same contract as the reference's ``src/orion/core/io/database/`` (``AbstractDB`` :23-264,
``EphemeralDB`` ephemeraldb.py:18-480, ``PickledDB`` pickleddb.py:29-207, ``MongoDB``
mongodb.py:30-295): ``write`` (insert, or ``$set`` update with a query), ``read`` (query +
projection), ``read_and_write`` (atomic find-and-modify of the first match), ``count``,
``remove``, ``ensure_index`` (unique indexes raise :class:`DuplicateKeyError`),
``index_information`` and ``drop_index``.

Backends:
  * :class:`EphemeralDB` -- in-process, for ``--debug`` and tests.  Documents are stored nested
    with an ``_id`` hash index, so ``read_and_write`` by id and unique checks are O(1) instead of
    the reference's flattened linear scans.
  * :class:`PickledDB` -- an EphemeralDB persisted in one file, every operation under a
    ``FileLock`` with an atomic tmp-file + rename write, for workers on a shared filesystem.
  * :class:`MongoDB` -- pymongo, ``find_one_and_update`` for the atomic reserve.

Query operators: equality on dotted keys, ``$ne $in $nin $gt $gte $lt $lte $exists``.
"""
from __future__ import annotations


import copy
import datetime
import logging
import os
import pickle
from contextlib import contextmanager
from typing import Any, Dict, Iterable, List, Optional

from ..utils.registry import Registry


_ATOMIC = (str, int, float, bool, type(None), bytes, datetime.datetime, datetime.date)


def _copy_doc(value):
    """Deep copy of a JSON/BSON-like document (dicts, lists, tuples, scalars, datetimes):
    several times faster than ``copy.deepcopy`` (no memo, no reduce protocol), which matters
    because every insert/read/update of the in-memory backends copies documents."""
    t = type(value)
    if t is dict:
        return {k: _copy_doc(v) for k, v in value.items()}
    if t is list:
        return [_copy_doc(v) for v in value]
    if t in _ATOMIC or isinstance(value, _ATOMIC):
        return value
    if t is tuple:
        return tuple(_copy_doc(v) for v in value)
    return copy.deepcopy(value)

log = logging.getLogger(__name__)
logging.getLogger("filelock").setLevel("ERROR")


class DatabaseError(RuntimeError):
    """Backend-independent database failure."""


class DuplicateKeyError(DatabaseError):
    """A write would duplicate a unique index value."""


class OutdatedDatabaseError(DatabaseError):
    """The database schema is older than this version of the framework (run ``db upgrade``)."""


class DatabaseTimeout(DatabaseError):
    """The database lock or server could not be acquired in time."""


DATABASES = Registry("Database")


# ----------------------------------------------------------------------------------------------
# Query / projection engine on nested documents
# ----------------------------------------------------------------------------------------------
_MISSING = object()
_NO_HASH_INDEX = ("_id", "results", "start_time", "end_time", "submit_time", "heartbeat")


def _get_path(doc, key: str):
    if "." not in key:                      # top-level field: the common case
        if isinstance(doc, dict):
            return doc.get(key, _MISSING)
        return _MISSING
    cur = doc
    for part in key.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        elif isinstance(cur, list) and part.isdigit() and int(part) < len(cur):
            cur = cur[int(part)]
        else:
            return _MISSING
    return cur


def _cmp(op, a, b):
    try:
        return op(a, b)
    except TypeError:
        return False


_OPS = {
    "$ne": lambda a, b: a is _MISSING or a != b,
    "$in": lambda a, b: a is not _MISSING and a in b,
    "$nin": lambda a, b: a is _MISSING or a not in b,
    "$gt": lambda a, b: a is not _MISSING and a is not None and _cmp(lambda x, y: x > y, a, b),
    "$gte": lambda a, b: a is not _MISSING and a is not None and _cmp(lambda x, y: x >= y, a, b),
    "$lt": lambda a, b: a is not _MISSING and a is not None and _cmp(lambda x, y: x < y, a, b),
    "$lte": lambda a, b: a is not _MISSING and a is not None and _cmp(lambda x, y: x <= y, a, b),
    "$exists": lambda a, b: (a is not _MISSING) == bool(b),
}


def _flatten_query(query: dict, prefix: str = "") -> List[tuple]:
    """-> [(dotted_key, op, value)]; nested non-operator dicts become dotted keys."""
    out = []
    for k, v in query.items():
        key = f"{prefix}.{k}" if prefix else k
        if isinstance(v, dict) and v and all(str(x).startswith("$") for x in v):
            for op, val in v.items():
                if op not in _OPS:
                    raise ValueError(f"Operator '{op}' is not supported")
                out.append((key, op, val))
        elif isinstance(v, dict) and v:
            out.extend(_flatten_query(v, key))
        elif k.split(".")[-1].startswith("$"):
            parts = key.split(".")
            op = parts[-1]
            if op not in _OPS:
                raise ValueError(f"Operator '{op}' is not supported")
            out.append((".".join(parts[:-1]), op, v))
        else:
            out.append((key, "$eq", v))
    return out


def match(doc: dict, query: Optional[dict]) -> bool:
    if not query:
        return True
    return _match_flat(doc, _flatten_query(query))


def _match_flat(doc: dict, flat: List[tuple]) -> bool:
    """:func:`match` against an already flattened query (scans flatten it once)."""
    for key, op, val in flat:
        cur = _get_path(doc, key)
        if op == "$eq":
            if cur is _MISSING or cur != val:
                return False
        elif not _OPS[op](cur, val):
            return False
    return True


def _set_path(doc, key: str, value, cow: bool = False):
    """Set a dotted key; with ``cow`` every dict on the path is shallow-copied first, so a
    shallow copy of a document can be updated without touching the original's nested dicts."""
    parts = key.split(".")
    cur = doc
    for p in parts[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
        elif cow:
            nxt = dict(nxt)
        cur[p] = nxt
        cur = nxt
    cur[parts[-1]] = value


def apply_update(doc: dict, data: dict, cow: bool = False) -> None:
    """``$set`` (default when no operator is given), ``$inc``, ``$unset``, ``$push``."""
    if any(k.startswith("$") for k in data):
        for op, fields in data.items():
            for key, value in _flatten_set(fields).items():
                if op == "$set":
                    _set_path(doc, key, _copy_doc(value), cow)
                elif op == "$inc":
                    cur = _get_path(doc, key)
                    _set_path(doc, key, (0 if cur is _MISSING or cur is None else cur) + value)
                elif op == "$unset":
                    parts = key.split(".")
                    parent = _get_path(doc, ".".join(parts[:-1])) if len(parts) > 1 else doc
                    if isinstance(parent, dict):
                        parent.pop(parts[-1], None)
                elif op == "$push":
                    cur = _get_path(doc, key)
                    _set_path(doc, key, ([] if cur is _MISSING or cur is None else list(cur))
                              + [_copy_doc(value)])
                else:
                    raise ValueError(f"Update operator '{op}' is not supported")
    else:
        for key, value in _flatten_set(data).items():
            _set_path(doc, key, _copy_doc(value), cow)


def _flatten_set(fields: dict) -> dict:
    """Dotted keys for nested dicts given to $set, but keep dict *values* of dotted keys whole."""
    out = {}
    for k, v in fields.items():
        out[k] = v
    return out


def project(doc: dict, selection: Optional[dict]) -> dict:
    """Mongo-style projection: all-1 (include) or all-0 (exclude); ``_id`` shown unless 0."""
    if not selection:
        return _copy_doc(doc)
    sel = dict(selection)
    id_flag = sel.pop("_id", 1)
    if sel:
        flags = set(bool(v) for v in sel.values())
        if len(flags) > 1:
            raise ValueError(f"Cannot mix selection with 1 and 0s except for _id: {selection}")
        include = flags.pop()
    else:
        include = bool(id_flag)
        if include:
            return {"_id": _copy_doc(doc.get("_id"))} if "_id" in doc else {}
        out = _copy_doc(doc)
        out.pop("_id", None)
        return out
    if include:
        out: Dict[str, Any] = {}
        for key in sel:
            val = _get_path(doc, key)
            _set_path(out, key, None if val is _MISSING else _copy_doc(val))
        if id_flag and "_id" in doc:
            out["_id"] = _copy_doc(doc["_id"])
        return out
    out = _copy_doc(doc)
    for key in sel:
        parts = key.split(".")
        parent = _get_path(out, ".".join(parts[:-1])) if len(parts) > 1 else out
        if isinstance(parent, dict):
            parent.pop(parts[-1], None)
    if not id_flag:
        out.pop("_id", None)
    return out


def index_name(keys) -> str:
    """Mongo-style index names: ``_id_`` or ``name_1_version_1``."""
    if not isinstance(keys, (list, tuple)):
        keys = [(keys, 1)]
    names = [k if isinstance(k, str) else k[0] for k in keys]
    if names == ["_id"]:
        return "_id_"
    orders = [1 if isinstance(k, str) else (1 if k[1] in (1, AbstractDB.ASCENDING) else -1)
              for k in keys]
    return "_".join(f"{n}_{o}" for n, o in zip(names, orders))


def _touched_keys(data) -> set:
    """Top-level document keys an update writes (``$set``-style dotted keys included)."""
    keys = set()
    for k, v in data.items():
        if k.startswith("$") and isinstance(v, dict):
            keys |= {kk.split(".", 1)[0] for kk in v}
        else:
            keys.add(k.split(".", 1)[0])
    return keys


def _affected(fields, touched) -> bool:
    if touched is None:
        return True
    for f in fields:
        if (f if "." not in f else f.split(".", 1)[0]) in touched:
            return True
    return False


def _hashable(v):
    if type(v) in _ATOMIC:
        return v
    if isinstance(v, dict):
        return tuple(sorted((k, _hashable(x)) for k, x in v.items()))
    if isinstance(v, (list, tuple)):
        return tuple(_hashable(x) for x in v)
    return v


# ----------------------------------------------------------------------------------------------
# Interfaces
# ----------------------------------------------------------------------------------------------
class AbstractDB:
    ASCENDING = 0
    DESCENDING = 1

    def __init__(self, host="localhost", name=None, port=None, username=None, password=None,
                 **kwargs):
        self.host = host
        self.name = name
        self.port = port
        self.username = username
        self.password = password
        self.options = kwargs
        self._db = None
        self._conn = None
        self.initiate_connection()

    @property
    def is_connected(self) -> bool:
        raise NotImplementedError

    def initiate_connection(self):
        raise NotImplementedError

    def close_connection(self):
        raise NotImplementedError

    def ensure_index(self, collection_name, keys, unique=False):
        raise NotImplementedError

    def index_information(self, collection_name) -> dict:
        raise NotImplementedError

    def drop_index(self, collection_name, name):
        raise NotImplementedError

    def write(self, collection_name, data, query=None) -> int:
        raise NotImplementedError

    def read(self, collection_name, query=None, selection=None) -> List[dict]:
        raise NotImplementedError

    def read_and_write(self, collection_name, query, data, selection=None) -> Optional[dict]:
        raise NotImplementedError

    def count(self, collection_name, query=None) -> int:
        raise NotImplementedError

    def remove(self, collection_name, query) -> int:
        raise NotImplementedError

    @property
    def configuration(self) -> dict:
        return {"type": type(self).__name__.lower(), "host": self.host, "name": self.name}


class ReadOnlyDB:
    """Read-only view (``read``/``count`` only) handed to experiment views."""

    __slots__ = ("_database",)
    valid_attributes = ["host", "name", "port", "username", "password", "is_connected",
                        "initiate_connection", "close_connection", "read", "count"]

    def __init__(self, database):
        self._database = database

    def __getattr__(self, attr):
        if attr not in self.valid_attributes:
            raise AttributeError(f"Cannot access attribute {attr} on view-only experiments.")
        return getattr(self._database, attr)


# ----------------------------------------------------------------------------------------------
# In-memory backend
# ----------------------------------------------------------------------------------------------
class _Collection:
    """Documents by ``_id`` plus indexes: unique ones reject duplicates, every single-field index
    is also a hash index (value -> ids) that equality / ``$in`` queries use to avoid full scans."""

    def __init__(self):
        self.docs: Dict[Any, dict] = {}  # hashable _id -> doc (insertion-ordered)
        self.indexes: Dict[str, tuple] = {}  # name -> (fields, unique, set of values)
        self.hash_index: Dict[str, Dict[Any, set]] = {}  # field -> value -> set(hashable _id)
        self._next_id = 1
        self.create_index("_id", unique=True)

    def create_index(self, keys, unique=False):
        if not isinstance(keys, (list, tuple)):
            keys = [(keys, AbstractDB.ASCENDING)]
        keys = [(k, AbstractDB.ASCENDING) if isinstance(k, str) else tuple(k) for k in keys]
        name = index_name(keys)
        if name in self.indexes:
            return name
        fields = tuple(k for k, _ in keys)
        values = set()
        if unique:
            for d in self.docs.values():
                v = self._key(d, fields)
                if v in values:
                    raise DuplicateKeyError(f"Duplicate key error: index={name} value={v}")
                values.add(v)
        self.indexes[name] = (fields, unique, values)
        # hash index only for scalar fields queried by equality / $in ("results" holds a list of
        # result documents: hashing it on every update cost more than all other indexing; the
        # timestamps are only ever range-queried or sorted -- lost trials, stats -- which an
        # equality index never serves, while a device sweep rewrites them thousands of times per
        # second)
        if len(fields) == 1 and fields[0] not in _NO_HASH_INDEX and \
                fields[0] not in self.hash_index:
            hidx: Dict[Any, set] = {}
            for hid, d in self.docs.items():
                hidx.setdefault(self._hval(d, fields[0]), set()).add(hid)
            self.hash_index[fields[0]] = hidx
        return name

    # -- on-disk format (PickledDB pickles whole collections) ------------------------------------
    FORMAT = 2

    def __getstate__(self):
        return {"format": self.FORMAT, "docs": self.docs, "indexes": self.indexes,
                "hash_index": self.hash_index, "next_id": self._next_id}

    def __setstate__(self, state):
        """Load any layout this backend ever wrote.  Format 2 is stored as built (a load costs
        one unpickle, no re-indexing).  Anything else -- the first release's bare ``__dict__``,
        indexes keyed by their field tuple (the index signature the reference changed in
        v0.1.6) or missing hash indexes -- is re-indexed from the documents and flagged
        ``migrated`` so ``mopt db upgrade`` rewrites it."""
        self.docs = state["docs"]
        self._next_id = state.get("next_id", state.get("_next_id", 1))
        self.migrated = state.get("format") != self.FORMAT
        if not self.migrated:
            self.indexes = state["indexes"]
            self.hash_index = state["hash_index"]
            return
        self.indexes, self.hash_index = {}, {}
        for name, spec in state.get("indexes", {}).items():
            fields = tuple(spec[0]) if isinstance(name, str) else tuple(name)
            unique = bool(spec[1]) if isinstance(spec, tuple) and len(spec) > 1 else True
            self.create_index([(f, AbstractDB.ASCENDING) for f in fields], unique=unique)
        if "_id_" not in self.indexes:
            self.create_index("_id", unique=True)

    def drop_index(self, name):
        fields, _, _ = self.indexes.pop(name)
        if len(fields) == 1 and not any(f == fields for f, _, _ in self.indexes.values()):
            self.hash_index.pop(fields[0], None)

    @staticmethod
    def _hval(doc, field):
        v = _get_path(doc, field)
        try:
            return _hashable(None if v is _MISSING else v)
        except TypeError:  # pragma: no cover - unhashable leaf
            return repr(v)

    @staticmethod
    def _key(doc, fields):
        return tuple(_hashable(None if (v := _get_path(doc, f)) is _MISSING else v)
                     for f in fields)

    def _check_unique(self, doc, touched=None):
        for name, (fields, unique, values) in self.indexes.items():
            if unique and _affected(fields, touched) and self._key(doc, fields) in values:
                raise DuplicateKeyError(f"Duplicate key error: index={name} "
                                        f"value={self._key(doc, fields)}")

    def _register(self, doc, touched=None):
        """Add ``doc`` to the indexes (only those over a top-level key in ``touched``, if given:
        an update re-indexes just what it changed)."""
        hid = _hashable(doc["_id"])
        for fields, unique, values in self.indexes.values():
            if unique and _affected(fields, touched):
                values.add(self._key(doc, fields))
        for field, hidx in self.hash_index.items():
            if _affected((field,), touched):
                hidx.setdefault(self._hval(doc, field), set()).add(hid)

    def _unregister(self, doc, touched=None):
        hid = _hashable(doc["_id"])
        for fields, unique, values in self.indexes.values():
            if unique and _affected(fields, touched):
                values.discard(self._key(doc, fields))
        for field, hidx in self.hash_index.items():
            if _affected((field,), touched):
                s = hidx.get(self._hval(doc, field))
                if s is not None:
                    s.discard(hid)

    def insert(self, doc: dict):
        if "_id" not in doc:
            while self._next_id in self.docs:
                self._next_id += 1
            doc["_id"] = self._next_id
            self._next_id += 1
        stored = _copy_doc(doc)
        self._check_unique(stored)
        self.docs[_hashable(stored["_id"])] = stored
        self._register(stored)

    def _candidates(self, query):
        """Ids narrowed by the most selective hash-indexed equality / $in clause, or None."""
        best = None
        for key, val in query.items():
            if key not in self.hash_index:
                continue
            hidx = self.hash_index[key]
            if isinstance(val, dict):
                if set(val) == {"$in"}:
                    ids = set()
                    for v in val["$in"]:
                        ids |= hidx.get(_hashable(v), set())
                else:
                    continue
            else:
                try:
                    ids = hidx.get(_hashable(val), set())
                except TypeError:  # pragma: no cover
                    continue
            if best is None or len(ids) < len(best):
                best = ids
        return best

    def find_iter(self, query):
        if query and "_id" in query and not isinstance(query["_id"], dict):
            # primary-key lookup, then the other clauses (compare-and-swap updates)
            d = self.docs.get(_hashable(query["_id"]))
            if d is None or (len(query) > 1 and not match(d, query)):
                return []
            return [d]
        if query:
            cands = self._candidates(query)
            if cands is not None:
                # keep insertion order for deterministic "first match" semantics
                if len(cands) * 8 < len(self.docs):
                    docs = sorted((self.docs[i] for i in cands if i in self.docs),
                                  key=lambda d: self._order(d))
                else:
                    docs = [d for i, d in self.docs.items() if i in cands]
                flat = _flatten_query(query)
                return [d for d in docs if _match_flat(d, flat)]
            flat = _flatten_query(query)
            return [d for d in self.docs.values() if _match_flat(d, flat)]
        return list(self.docs.values())

    def _order(self, doc):
        if not hasattr(self, "_pos") or len(self._pos) != len(self.docs):
            self._pos = {k: i for i, k in enumerate(self.docs)}
        return self._pos.get(_hashable(doc["_id"]), 0)

    def update(self, doc: dict, data: dict):
        new = dict(doc)                  # copy-on-write: untouched sub-documents are shared
        apply_update(new, data, cow=True)
        if new.get("_id") != doc.get("_id"):
            raise DatabaseError("cannot change _id")
        touched = _touched_keys(data)
        self._unregister(doc, touched)
        try:
            self._check_unique(new, touched)
        except DuplicateKeyError:
            self._register(doc, touched)
            raise
        doc.clear()
        doc.update(new)
        self._register(doc, touched)

    def delete(self, doc):
        self._unregister(doc)
        del self.docs[_hashable(doc["_id"])]

    def insert_owned(self, docs) -> int:
        """Bulk insert of documents the caller hands over (no defensive copy).

        Indexes over top-level fields only (every index the storage creates) are maintained
        inline -- one dict lookup per indexed field instead of the dotted-path machinery of
        :meth:`_register`: this is the write path of a device sweep's thousands of trials per
        second (worker/writer.py)."""
        uniq = [(fields, values) for fields, unique, values in self.indexes.values() if unique]
        hashed = list(self.hash_index.items())
        if any("." in f for fields, _ in uniq for f in fields) or \
                any("." in f for f, _ in hashed):
            for d in docs:
                if "_id" not in d:
                    self.insert(d)
                    continue
                self._check_unique(d)
                self.docs[_hashable(d["_id"])] = d
                self._register(d)
            return len(docs)
        store, atomic = self.docs, _ATOMIC
        for d in docs:
            if "_id" not in d:
                self.insert(d)
                continue
            keys = []
            for fields, values in uniq:
                k = tuple(v if type(v := d.get(f)) in atomic else _hashable(v) for f in fields)
                if k in values:
                    raise DuplicateKeyError(f"Duplicate key error: fields={fields} value={k}")
                keys.append(k)
            hid = _hashable(d["_id"])
            store[hid] = d
            for (_, values), k in zip(uniq, keys):
                values.add(k)
            for f, hidx in hashed:
                v = d.get(f)
                hv = v if type(v) in atomic else self._hval(d, f)
                ids = hidx.get(hv)
                if ids is None:
                    hidx[hv] = {hid}
                else:
                    ids.add(hid)
        return len(docs)

    def set_fields_by_id(self, items, owned: bool = False) -> int:
        """Bulk ``$set`` of top-level fields: ``items`` = [(id, {field: value}, status or None)],
        each applied only while the document's status equals the given one (compare-and-swap).
        Same result as :meth:`update` per item without the generic operator machinery.
        ``owned``: the caller never touches the field values again (no defensive copy)."""
        uniq = {f for fields, unique, _ in self.indexes.values() if unique for f in fields}
        n = 0
        for uid, fields, was in items:
            hid = _hashable(uid)
            d = self.docs.get(hid)
            if d is None or (was is not None and d.get("status") != was):
                continue
            if "_id" in fields or uniq.intersection(fields):
                self.update(d, fields)     # unique-indexed field: the checked generic path
                n += 1
                continue
            for f, hidx in self.hash_index.items():
                if f in fields:
                    ids = hidx.get(self._hval(d, f))
                    if ids is not None:
                        ids.discard(hid)
            d.update(fields if owned else _copy_doc(fields))
            for f, hidx in self.hash_index.items():
                if f in fields:
                    hidx.setdefault(self._hval(d, f), set()).add(hid)
            n += 1
        return n


@DATABASES.register("ephemeraldb")
class EphemeralDB(AbstractDB):
    """Non-persistent in-process database (``--debug``; tests)."""

    @property
    def is_connected(self):
        return self._db is not None

    def initiate_connection(self):
        if self._db is None:
            self._db = {}

    def close_connection(self):
        pass

    def _col(self, name) -> _Collection:
        col = self._db.get(name)
        if col is None:
            col = self._db[name] = _Collection()
        return col

    def ensure_index(self, collection_name, keys, unique=False):
        self._col(collection_name).create_index(keys, unique=unique)

    def index_information(self, collection_name):
        return {name: unique for name, (_, unique, _) in self._col(collection_name).indexes.items()}

    def drop_index(self, collection_name, name):
        col = self._col(collection_name)
        if name not in col.indexes:
            raise DatabaseError(f"index not found with name {name}")
        col.drop_index(name)

    def write(self, collection_name, data, query=None):
        col = self._col(collection_name)
        if query is None:
            docs = data if isinstance(data, (list, tuple)) else [data]
            for d in docs:
                col.insert(d)
            return len(docs)
        n = 0
        for d in list(col.find_iter(query)):
            col.update(d, data)
            n += 1
        return n

    def read(self, collection_name, query=None, selection=None):
        return [project(d, selection) for d in self._col(collection_name).find_iter(query)]

    def insert_owned(self, collection_name, docs) -> int:
        """Insert documents the caller will never touch again (no copy): bulk writers."""
        return self._col(collection_name).insert_owned(list(docs))

    def read_owned(self, collection_name, query=None) -> List[dict]:
        """:meth:`read` without the defensive copies: the stored documents themselves, for a
        caller that only serialises them (the writer child's final hand-back)."""
        return list(self._col(collection_name).find_iter(query))

    def set_fields_by_id(self, collection_name, items, owned: bool = False) -> int:
        """Bulk compare-and-swap field updates by ``_id`` (see ``_Collection``)."""
        return self._col(collection_name).set_fields_by_id(items, owned)

    def read_and_write(self, collection_name, query, data, selection=None):
        col = self._col(collection_name)
        found = col.find_iter(query)
        if not found:
            return None
        doc = found[0]
        col.update(doc, data)
        return project(doc, selection)

    def count(self, collection_name, query=None):
        col = self._col(collection_name)
        if not query:
            return len(col.docs)
        return len(col.find_iter(query))

    def remove(self, collection_name, query):
        col = self._col(collection_name)
        found = list(col.find_iter(query))
        for d in found:
            col.delete(d)
        return len(found)

    def drop(self, collection_name):
        self._db.pop(collection_name, None)

    def collection_names(self):
        return sorted(self._db)


# ----------------------------------------------------------------------------------------------
# File backend
# ----------------------------------------------------------------------------------------------
def default_pickled_path() -> str:
    base = os.environ.get("XDG_DATA_HOME") or os.path.join(os.path.expanduser("~"), ".local",
                                                           "share")
    return os.path.join(base, "mopt", "mopt_db.pkl")


@DATABASES.register("pickleddb")
class PickledDB(AbstractDB):
    """An :class:`EphemeralDB` pickled to ``host`` (a file path), every op under a file lock.

    Collections pickle as format 2 (documents and built indexes, unpickled as stored);
    older files load through ``_Collection.__setstate__`` and are rewritten in the current
    format by the next write or by :meth:`upgrade_format` (``mopt db upgrade``)."""

    def upgrade_format(self) -> int:
        """Rewrite the file in the current format; returns how many collections were in an
        older one."""
        with self.locked_database() as db:
            return sum(1 for col in (db._db or {}).values() if getattr(col, "migrated", False))

    LOCK_TIMEOUT = 60

    def __init__(self, host=None, name=None, *args, timeout=None, **kwargs):
        host = host or default_pickled_path()
        if host in ("localhost", ""):
            host = default_pickled_path()
        self.timeout = timeout if timeout is not None else self.LOCK_TIMEOUT
        super().__init__(host, name=name)
        d = os.path.dirname(os.path.abspath(host))
        os.makedirs(d, exist_ok=True)

    @property
    def is_connected(self):
        return True

    def initiate_connection(self):
        pass

    def close_connection(self):
        pass

    def _load(self) -> EphemeralDB:
        if not os.path.exists(self.host):
            return EphemeralDB()
        with open(self.host, "rb") as f:
            data = f.read()
        if not data:
            return EphemeralDB()
        return pickle.loads(data)  # our own file format, written by _dump below

    def _dump(self, db: EphemeralDB) -> None:
        tmp = f"{self.host}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            pickle.dump(db, f, protocol=pickle.HIGHEST_PROTOCOL)
        os.replace(tmp, self.host)

    @contextmanager
    def locked_database(self, write=True):
        from filelock import FileLock, Timeout
        lock = FileLock(self.host + ".lock")
        try:
            with lock.acquire(timeout=self.timeout):
                db = self._load()
                yield db
                if write:
                    self._dump(db)
        except Timeout as exc:
            raise DatabaseTimeout(f"could not acquire lock for PickledDB after {self.timeout} "
                                  "seconds") from exc

    def ensure_index(self, collection_name, keys, unique=False):
        with self.locked_database() as db:
            db.ensure_index(collection_name, keys, unique=unique)

    def index_information(self, collection_name):
        with self.locked_database(write=False) as db:
            return db.index_information(collection_name)

    def drop_index(self, collection_name, name):
        with self.locked_database() as db:
            return db.drop_index(collection_name, name)

    def write(self, collection_name, data, query=None):
        with self.locked_database() as db:
            return db.write(collection_name, data, query=query)

    def read(self, collection_name, query=None, selection=None):
        with self.locked_database(write=False) as db:
            return db.read(collection_name, query=query, selection=selection)

    def read_and_write(self, collection_name, query, data, selection=None):
        with self.locked_database() as db:
            return db.read_and_write(collection_name, query, data, selection=selection)

    def count(self, collection_name, query=None):
        with self.locked_database(write=False) as db:
            return db.count(collection_name, query=query)

    def remove(self, collection_name, query):
        with self.locked_database() as db:
            return db.remove(collection_name, query)


# ----------------------------------------------------------------------------------------------
# MongoDB backend
# ----------------------------------------------------------------------------------------------
@DATABASES.register("mongodb")
class MongoDB(AbstractDB):
    """pymongo backend; ``host`` may be a ``mongodb://`` URI (user, password, db name parsed)."""

    def __init__(self, host="localhost", name=None, port=None, username=None, password=None,
                 serverSelectionTimeoutMS=5000, **kwargs):
        self._timeout_ms = serverSelectionTimeoutMS
        if host and str(host).startswith("mongodb://"):
            from pymongo.uri_parser import parse_uri
            info = parse_uri(host)
            username = username or info.get("username")
            password = password or info.get("password")
            name = name or info.get("database")
            port = port or (info["nodelist"][0][1] if info.get("nodelist") else None)
        super().__init__(host, name, port or 27017, username, password, **kwargs)

    @property
    def is_connected(self):
        return self._conn is not None

    def initiate_connection(self):
        if self._conn is not None:
            return
        import pymongo
        from pymongo.errors import ConnectionFailure, OperationFailure
        try:
            self._conn = pymongo.MongoClient(
                host=self.host, port=int(self.port) if self.port else None,
                username=self.username, password=self.password,
                serverSelectionTimeoutMS=self._timeout_ms)
            self._db = self._conn[self.name or "mopt"]
            self._conn.admin.command("ping")
        except (ConnectionFailure, OperationFailure) as exc:
            self._conn = None
            raise DatabaseError(str(exc)) from exc

    def close_connection(self):
        if self._conn is not None:
            self._conn.close()
            self._conn = None

    @contextmanager
    def _errors(self):
        from pymongo import errors
        try:
            yield
        except errors.DuplicateKeyError as exc:
            raise DuplicateKeyError(str(exc)) from exc
        except errors.BulkWriteError as exc:
            raise DuplicateKeyError(str(exc)) from exc
        except (errors.ConnectionFailure, errors.OperationFailure) as exc:
            raise DatabaseError(str(exc)) from exc

    def ensure_index(self, collection_name, keys, unique=False):
        import pymongo
        if not isinstance(keys, (list, tuple)):
            keys = [(keys, self.ASCENDING)]
        keys = [(k, pymongo.ASCENDING if o == self.ASCENDING else pymongo.DESCENDING)
                for k, o in keys]
        with self._errors():
            self._db[collection_name].create_index(keys, unique=unique, background=True)

    def index_information(self, collection_name):
        with self._errors():
            info = self._db[collection_name].index_information()
        return {name: info[name].get("unique", name == "_id_") for name in info}

    def drop_index(self, collection_name, name):
        with self._errors():
            self._db[collection_name].drop_index(name)

    @staticmethod
    def _query(query):
        """Queries as the in-memory backends read them: a nested plain dict matches fields of a
        sub-document (``{'meta': {'user': 'u'}}`` == ``{'meta.user': 'u'}``) instead of
        MongoDB's whole-embedded-document equality, so every backend answers alike."""
        if not query:
            return {}
        out = {}
        for key, op, val in _flatten_query(query):
            if op == "$eq":
                out[key] = val
            else:
                out.setdefault(key, {})[op] = val
        return out

    @staticmethod
    def _selection(selection):
        if selection:
            sel = {k: v for k, v in selection.items() if k != "_id"}
            if len(set(bool(v) for v in sel.values())) > 1:
                raise ValueError("Cannot mix selection with 1 and 0s except for _id: "
                                 f"{selection}")
        return selection

    def write(self, collection_name, data, query=None):
        col = self._db[collection_name]
        with self._errors():
            if query is None:
                docs = data if isinstance(data, (list, tuple)) else [data]
                res = col.insert_many(docs)
                return len(res.inserted_ids)
            update = data if any(k.startswith("$") for k in data) else {"$set": data}
            return col.update_many(self._query(query), update).modified_count

    def read(self, collection_name, query=None, selection=None):
        selection = self._selection(selection)
        with self._errors():
            return list(self._db[collection_name].find(self._query(query), selection))

    def read_and_write(self, collection_name, query, data, selection=None):
        import pymongo
        update = data if any(k.startswith("$") for k in data) else {"$set": data}
        with self._errors():
            return self._db[collection_name].find_one_and_update(
                self._query(query), update, projection=self._selection(selection),
                return_document=pymongo.ReturnDocument.AFTER)

    def count(self, collection_name, query=None):
        with self._errors():
            return self._db[collection_name].count_documents(self._query(query))

    def remove(self, collection_name, query):
        with self._errors():
            return self._db[collection_name].delete_many(self._query(query)).deleted_count


def create_database(of_type: str = "ephemeraldb", **config) -> AbstractDB:
    """Instantiate a backend by (case-insensitive) name."""
    cls = DATABASES.get(of_type)
    config = {k: v for k, v in config.items() if v is not None}
    return cls(**config)
