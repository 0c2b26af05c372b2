"""A small in-memory stand-in for the parts of ``pymongo`` the MongoDB backend uses, so the
database and storage-protocol contract tests run against ``MongoDB`` without a server
(reference: tests/unittests/core/mongodb_test.py needs a live MongoDB).

Its query matching, projections and updates are written independently of ``EphemeralDB`` --
following MongoDB's documented semantics -- so the contract suite compares two
implementations, not one implementation with itself.  Install with :func:`install`.
"""
from __future__ import annotations

import copy
import itertools
import sys
import types
from urllib.parse import unquote, urlparse

ASCENDING, DESCENDING = 1, -1
_ids = itertools.count(1)


class ReturnDocument:
    BEFORE, AFTER = False, True


class _errors(types.ModuleType):
    class PyMongoError(Exception):
        pass

    class ConnectionFailure(PyMongoError):
        pass

    class OperationFailure(PyMongoError):
        pass

    class DuplicateKeyError(OperationFailure):
        pass

    class BulkWriteError(OperationFailure):
        pass


errors = _errors("pymongo.errors")
_MISSING = object()


def _get(doc, path):
    cur = doc
    for part in path.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        else:
            return _MISSING
    return cur


def _cond(value, cond):
    if isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond):
        for op, arg in cond.items():
            present = value is not _MISSING
            if op == "$ne" and present and value == arg:
                return False
            if op == "$in" and not (present and value in arg):
                return False
            if op == "$nin" and present and value in arg:
                return False
            if op in ("$gt", "$gte", "$lt", "$lte"):
                if not present or value is None:
                    return False
                ok = {"$gt": value > arg, "$gte": value >= arg,
                      "$lt": value < arg, "$lte": value <= arg}[op]
                if not ok:
                    return False
            if op == "$exists" and present != bool(arg):
                return False
        return True
    return (None if value is _MISSING else value) == cond


def _match(doc, query):
    return all(_cond(_get(doc, k), v) for k, v in (query or {}).items())


def _project(doc, selection):
    if not selection:
        return copy.deepcopy(doc)
    include = {k for k, v in selection.items() if v}
    if include:
        out = {}
        for k in include | {"_id"}:
            if selection.get(k, 1) == 0:
                continue
            v = _get(doc, k)
            if v is not _MISSING:
                cur = out
                parts = k.split(".")
                for p in parts[:-1]:
                    cur = cur.setdefault(p, {})
                cur[parts[-1]] = copy.deepcopy(v)
        return out
    out = copy.deepcopy(doc)
    for k, v in selection.items():
        if not v:
            out.pop(k, None)
    return out


def _set(doc, path, value):
    parts = path.split(".")
    cur = doc
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = copy.deepcopy(value)


class _Result:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class Collection:
    def __init__(self):
        self.docs = []
        self.indexes = {"_id_": ((("_id", 1),), True)}

    def _check(self, doc, skip=None):
        for name, (keys, unique) in self.indexes.items():
            if not unique:
                continue
            key = tuple(repr(_get(doc, k)) for k, _ in keys)
            for other in self.docs:
                if other is skip or other is doc:
                    continue
                if tuple(repr(_get(other, k)) for k, _ in keys) == key:
                    raise errors.DuplicateKeyError(f"E11000 duplicate key {name} {key}")

    def insert_many(self, docs):
        ids = []
        for d in docs:
            d.setdefault("_id", next(_ids))     # pymongo sets _id on the caller's document
            d = copy.deepcopy(d)
            try:
                self._check(d)
            except errors.DuplicateKeyError as exc:
                raise errors.BulkWriteError(str(exc)) from exc
            self.docs.append(d)
            ids.append(d["_id"])
        return _Result(inserted_ids=ids)

    def find(self, query=None, projection=None):
        return [_project(d, projection) for d in self.docs if _match(d, query)]

    def _apply(self, doc, update):
        new = copy.deepcopy(doc)
        for op, fields in update.items():
            if op == "$set":
                for k, v in fields.items():
                    _set(new, k, v)
            elif op == "$inc":                  # MongoDB: a missing field counts as 0
                for k, v in fields.items():
                    cur = _get(new, k)
                    _set(new, k, (0 if cur is _MISSING else cur) + v)
            else:
                raise errors.OperationFailure(f"unsupported update operator {op}")
        self._check(new, skip=doc)
        doc.clear()
        doc.update(new)

    def update_many(self, query, update):
        n = 0
        for d in [d for d in self.docs if _match(d, query)]:
            self._apply(d, update)
            n += 1
        return _Result(modified_count=n, matched_count=n)

    def find_one_and_update(self, query, update, projection=None, return_document=False):
        for d in self.docs:
            if _match(d, query):
                before = copy.deepcopy(d)
                self._apply(d, update)
                return _project(d if return_document else before, projection)
        return None

    def count_documents(self, query):
        return sum(1 for d in self.docs if _match(d, query))

    def delete_many(self, query):
        keep = [d for d in self.docs if not _match(d, query)]
        n = len(self.docs) - len(keep)
        self.docs = keep
        return _Result(deleted_count=n)

    def create_index(self, keys, unique=False, background=False):
        keys = tuple((k, o) for k, o in keys)
        name = "_".join(f"{k}_{o}" for k, o in keys)
        self.indexes[name] = (keys, unique)
        if unique:
            for d in self.docs:
                self._check(d)
        return name

    def index_information(self):
        return {name: {"key": list(keys), "unique": unique}
                for name, (keys, unique) in self.indexes.items()}

    def drop_index(self, name):
        if name not in self.indexes:
            raise errors.OperationFailure(f"index not found with name [{name}]")
        del self.indexes[name]


class Database(dict):
    def __missing__(self, name):
        col = self[name] = Collection()
        return col


class _Admin:
    def command(self, name):
        return {"ok": 1}


SERVERS: dict = {}          # (host, port) -> {db name: Database}


class MongoClient:
    def __init__(self, host="localhost", port=None, username=None, password=None,
                 serverSelectionTimeoutMS=None, **kw):
        if str(host).startswith("mongodb://unreachable"):
            raise errors.ConnectionFailure("No servers found yet")
        self.key = (host, port)
        self.server = SERVERS.setdefault(self.key, {})
        self.admin = _Admin()

    def __getitem__(self, name):
        return self.server.setdefault(name, Database())

    def close(self):
        pass


def _parse_uri(uri):
    u = urlparse(uri)
    return {"username": unquote(u.username) if u.username else None,
            "password": unquote(u.password) if u.password else None,
            "database": u.path.lstrip("/") or None,
            "nodelist": [(u.hostname, u.port or 27017)]}


def install(monkeypatch):
    """Make ``import pymongo`` resolve to this module for the duration of a test."""
    mod = sys.modules[__name__]
    uri_parser = types.ModuleType("pymongo.uri_parser")
    uri_parser.parse_uri = _parse_uri
    mod.uri_parser = uri_parser
    mod.errors = errors
    monkeypatch.setitem(sys.modules, "pymongo", mod)
    monkeypatch.setitem(sys.modules, "pymongo.errors", errors)
    monkeypatch.setitem(sys.modules, "pymongo.uri_parser", uri_parser)
    SERVERS.clear()
