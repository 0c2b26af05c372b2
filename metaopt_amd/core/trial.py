"""The trial document (reference: ``src/orion/core/worker/trial.py:18-334``).

Byte-compatible ``to_dict`` schema::

    {_id, experiment, status, worker, heartbeat, submit_time, start_time, end_time,
     results: [{name, type, value}], params: [{name, type, value}], parents: [...]}

``_id`` is the md5 of ``params_repr + str(experiment) + lie_repr``: the deduplication key shared
by every worker (host or device) registering trials in one experiment.
"""
from __future__ import annotations

import hashlib
import logging
from typing import List, Optional

log = logging.getLogger(__name__)


class Value:
    __slots__ = ("name", "_type", "value")
    allowed_types: tuple = ()

    def __init__(self, name=None, type=None, value=None, **extra):  # noqa: A002
        self.name = name
        self._type = None
        self.type = type
        if hasattr(value, "tolist"):  # numpy scalars/arrays -> plain python
            value = value.tolist()
        self.value = value

    def to_dict(self):
        return {"name": self.name, "type": self.type, "value": self.value}

    def __eq__(self, other):
        return (isinstance(other, Value) and self.name == other.name and self.type == other.type
                and self.value == other.value)

    def __repr__(self):
        return (f"{type(self).__name__}(name={self.name!r}, type={self.type!r}, "
                f"value={self.value!r})")

    @property
    def type(self):
        return self._type

    @type.setter
    def type(self, type_):
        if type_ is not None and type_ not in self.allowed_types:
            raise ValueError(f"Given type, {type_}, not one of: {self.allowed_types}")
        self._type = type_


class Result(Value):
    __slots__ = ()
    allowed_types = ("objective", "constraint", "gradient", "statistic", "lie")


class Param(Value):
    __slots__ = ()
    allowed_types = ("integer", "real", "categorical", "fidelity")


class Trial:
    """One evaluation of a point of the search space."""

    __slots__ = ("experiment", "_id_override", "_status", "worker", "_working_dir", "heartbeat",
                 "submit_time", "start_time", "end_time", "_results", "params", "parents")
    allowed_stati = ("new", "reserved", "suspended", "completed", "interrupted", "broken")
    Value = Value
    Result = Result
    Param = Param

    def __init__(self, **kwargs):
        for attr in self.__slots__:
            setattr(self, attr, [] if attr in ("_results", "params", "parents") else None)
        self._status = "new"
        kwargs.pop("_id", None)
        kwargs.pop("id", None)
        for attr, value in kwargs.items():
            if attr == "results":
                self._results = [v if isinstance(v, Result) else Result(**v) for v in value]
            elif attr == "params":
                self.params = [v if isinstance(v, Param) else Param(**v) for v in value]
            elif attr == "status":
                self.status = value
            elif attr == "working_dir":
                self._working_dir = value
            elif attr in self.__slots__:
                setattr(self, attr, value)
            else:
                raise AttributeError(f"Trial has no attribute '{attr}'")

    @classmethod
    def build(cls, entries) -> List["Trial"]:
        return [cls(**e) for e in entries]

    def to_dict(self) -> dict:
        return {
            "experiment": self.experiment,
            "status": self._status,
            "worker": self.worker,
            "heartbeat": self.heartbeat,
            "submit_time": self.submit_time,
            "start_time": self.start_time,
            "end_time": self.end_time,
            "results": [r.to_dict() for r in self._results],
            "params": [p.to_dict() for p in self.params],
            "parents": list(self.parents),
            "_id": self.id,
        }

    def __str__(self):
        return (f"Trial(experiment={self.experiment!r}, status={self._status!r}, "
                f"params={self.params_repr()})")

    __repr__ = __str__

    # -- results ------------------------------------------------------------------------------
    @property
    def results(self) -> List[Result]:
        return self._results

    @results.setter
    def results(self, results):
        results = [r if isinstance(r, Result) else Result(**r) for r in results]
        objective = self._fetch_one(results, "objective")
        if objective is None:
            raise ValueError(f"No objective found in results: {results}")
        if not isinstance(objective.value, (float, int)) or isinstance(objective.value, bool):
            raise ValueError("Results must contain a type `objective` with type float/int: "
                             f"{objective}")
        self._results = results

    @property
    def objective(self) -> Optional[Result]:
        return self._fetch_one(self._results, "objective")

    @property
    def lie(self) -> Optional[Result]:
        return self._fetch_one(self._results, "lie")

    @property
    def gradient(self) -> Optional[Result]:
        return self._fetch_one(self._results, "gradient")

    @property
    def constraints(self) -> List[Result]:
        return [r for r in self._results if r.type == "constraint"]

    @property
    def statistics(self) -> List[Result]:
        return [r for r in self._results if r.type == "statistic"]

    @staticmethod
    def _fetch_one(results, rtype):
        vals = [r for r in results if r.type == rtype]
        if not vals:
            return None
        if len(vals) > 1:
            log.warning("Found multiple results of '%s' type; using the first: %s", rtype, vals[0])
        return vals[0]

    # -- identity -----------------------------------------------------------------------------
    @property
    def working_dir(self):
        return self._working_dir

    @working_dir.setter
    def working_dir(self, value):
        self._working_dir = value

    @property
    def status(self):
        return self._status

    @status.setter
    def status(self, status):
        if status is not None and status not in self.allowed_stati:
            raise ValueError(f"Given status, {status}, not one of: {self.allowed_stati}")
        self._status = status

    @staticmethod
    def _repr_values(values, sep=","):
        return sep.join(f"{v.name}:{v.value}" for v in values)

    def params_repr(self, sep=",") -> str:
        return self._repr_values(self.params, sep)

    @property
    def hash_name(self) -> str:
        if not self.params and not self.experiment:
            raise ValueError("Cannot distinguish this trial, as 'params' or 'experiment' "
                             "have not been set.")
        lie = self.lie
        lie_repr = self._repr_values([lie]) if lie else ""
        return hashlib.md5((self.params_repr() + str(self.experiment) + lie_repr)
                           .encode("utf-8")).hexdigest()

    @property
    def id(self) -> str:
        return self.hash_name

    def __hash__(self):
        return int(self.hash_name, 16)

    def __eq__(self, other):
        return isinstance(other, Trial) and self.to_dict() == other.to_dict()

    @property
    def full_name(self) -> str:
        if not self.params or not self.experiment:
            raise ValueError("Cannot distinguish this trial, as 'params' or 'experiment' "
                             "have not been set.")
        return self.params_repr(sep="-").replace("/", ".")

    @property
    def params_dict(self) -> dict:
        return {p.name: p.value for p in self.params}

    @property
    def arguments(self) -> dict:
        """Parameters without the leading '/' namespace (ROADMAP study API ``trial.arguments``)."""
        return {p.name.lstrip("/"): p.value for p in self.params}
