"""Adapters: how trials cross one edge of the experiment version-control tree.

Behaviour contract: ``src/orion/core/evc/adapters.py:45-869`` of the reference (which trials a
branch keeps, how their parameters are rewritten, the ``refers.adapter`` serialisation).  The
structure here is this package's own: every adapter is a *pair of per-trial rules* -- one per
direction -- drawn from a five-rule algebra, and the inverse of an adapter is the same pair
swapped.  A rule maps one trial to a (rewritten copy of the) trial or to ``None`` (dropped):

=================  =========================================================================
rule               effect on a trial
=================  =========================================================================
``insert(p)``      copy with parameter ``p`` added (the trial must not have ``p.name`` yet)
``strip_at(p)``    copy without ``p.name`` when its value equals ``p.value``, else dropped
``within(n, d)``   the trial itself when the value of ``n`` lies in dimension ``d``
``rename(a, b)``   copy with parameter ``a`` renamed ``b``
``keep`` / ``drop``  every trial / no trial
=================  =========================================================================

=====================  ======================  ========================
adapter                forward (parent->child)  backward (child->parent)
=====================  ======================  ========================
DimensionAddition      insert(p)                strip_at(p)
DimensionDeletion      strip_at(p)              insert(p)
DimensionPriorChange   within(n, new prior)     within(n, old prior)
DimensionRenaming      rename(old, new)         rename(new, old)
AlgorithmChange        keep                     keep
Code/CommandLine/      keep unless ``break``    keep only if ``noeffect``
ScriptConfig change
CompositeAdapter       members in order         members in reverse order
=====================  ======================  ========================

Serialisation: ``to_dict()`` gives ``{"of_type": <lower-case class name>, **fields}``;
``configuration`` is the list stored in a child's ``refers.adapter``; ``Adapter.build(list)``
rebuilds a :class:`CompositeAdapter` (nested lists become nested composites).
"""
from __future__ import annotations

import copy
from typing import Callable, Dict, List, Optional, Sequence

from ..core.trial import Param, Trial
from ..space.builder import DimensionBuilder

Rule = Callable[[Trial], Optional[Trial]]

_NOEFFECT, _BREAK, _UNSURE = "noeffect", "break", "unsure"
CHANGE_TYPES = (_NOEFFECT, _BREAK, _UNSURE)


# ---------------------------------------------------------------------------------- rule algebra
def _param_of(trial: Trial, name: str, must_exist: bool = True):
    for p in trial.params:
        if p.name == name:
            return p
    if must_exist:
        raise RuntimeError(f"trial {trial} cannot be adapted: its "
                           f"configuration has no dimension '{name}' (it should be present)")
    return None


def _with_params(trial: Trial, params) -> Trial:
    out = copy.deepcopy(trial)
    out.params = sorted(params, key=lambda p: p.name)
    return out


def insert(param: Param) -> Rule:
    def rule(trial):
        if _param_of(trial, param.name, must_exist=False) is not None:
            raise RuntimeError(f"cannot add dimension '{param.name}' to a trial where it is "
                               f"already present: {trial}")
        return _with_params(trial, list(copy.deepcopy(trial.params)) + [copy.deepcopy(param)])
    return rule


def strip_at(param: Param) -> Rule:
    def rule(trial):
        if _param_of(trial, param.name).value != param.value:
            return None
        return _with_params(trial, [copy.deepcopy(p) for p in trial.params
                                    if p.name != param.name])
    return rule


def within(name: str, dimension) -> Rule:
    def rule(trial):
        return trial if _param_of(trial, name).value in dimension else None
    return rule


def rename(old: str, new: str) -> Rule:
    def rule(trial):
        _param_of(trial, old)
        params = copy.deepcopy(trial.params)
        for p in params:
            if p.name == old:
                p.name = new
        return _with_params(trial, params)
    return rule


def keep(trial):
    return trial


def drop(trial):
    return None


def run_rule(rule: Rule, trials: Sequence[Trial]) -> List[Trial]:
    out = []
    for t in trials:
        r = rule(t)
        if r is not None:
            out.append(r)
    return out


# ---------------------------------------------------------------------------------- adapters
class BaseAdapter:
    """An edge adapter: ``forward`` (parent trials for the child) and ``backward``."""

    def _rules(self):
        """(forward rule, backward rule); composites override forward/backward instead."""
        raise NotImplementedError

    def forward(self, trials: List[Trial]) -> List[Trial]:
        return run_rule(self._rules()[0], trials)

    def backward(self, trials: List[Trial]) -> List[Trial]:
        return run_rule(self._rules()[1], trials)

    def _fields(self) -> dict:
        return {}

    def to_dict(self) -> dict:
        return {"of_type": type(self).__name__.lower(), **self._fields()}

    @property
    def configuration(self) -> list:
        return [self.to_dict()]

    def __eq__(self, other):
        return isinstance(other, BaseAdapter) and self.configuration == other.configuration

    def __repr__(self):
        return f"{type(self).__name__}({self._fields()})"


def _param(value) -> Param:
    if isinstance(value, Param):
        return value
    if isinstance(value, dict):
        return Param(**value)
    raise TypeError(f"expected a Param or a dict of Param fields (name, type, value), got "
                    f"{type(value).__name__}")


class DimensionAddition(BaseAdapter):
    """The child added a dimension: parents' trials get it at its default value; children's
    trials at that value flow back without it."""

    def __init__(self, param):
        self.param = _param(param)

    def _rules(self):
        return insert(self.param), strip_at(self.param)

    def _fields(self):
        return {"param": self.param.to_dict()}


class DimensionDeletion(DimensionAddition):
    """The child removed a dimension: the inverse of :class:`DimensionAddition`."""

    def _rules(self):
        fwd, bwd = super()._rules()
        return bwd, fwd


class DimensionPriorChange(BaseAdapter):
    """A dimension's prior changed: only trials inside the target prior cross the edge."""

    def __init__(self, name, old_prior, new_prior):
        self.name, self.old_prior, self.new_prior = name, old_prior, new_prior
        build = DimensionBuilder().build
        self._old = build("old", old_prior)
        self._new = build("new", new_prior)
        if self._old.shape != self._new.shape:
            raise NotImplementedError(f"prior of '{name}' changes shape ({self._old.shape} -> "
                                      f"{self._new.shape}): not adaptable")

    def _rules(self):
        return within(self.name, self._new), within(self.name, self._old)

    def _fields(self):
        return {"name": self.name, "old_prior": self.old_prior, "new_prior": self.new_prior}


class DimensionRenaming(BaseAdapter):
    def __init__(self, old_name, new_name):
        if not (isinstance(old_name, str) and isinstance(new_name, str)):
            raise TypeError("dimension names must be strings, got "
                            f"{type(old_name).__name__} and {type(new_name).__name__}")
        self.old_name, self.new_name = old_name, new_name

    def _rules(self):
        return rename(self.old_name, self.new_name), rename(self.new_name, self.old_name)

    def _fields(self):
        return {"old_name": self.old_name, "new_name": self.new_name}


class AlgorithmChange(BaseAdapter):
    """The algorithm changed: trials are still valid observations both ways."""

    def _rules(self):
        return keep, keep


class _ChangeKind(BaseAdapter):
    """A change outside the search space (code, command line, script configuration), typed by
    the user: ``noeffect`` (trials flow both ways), ``unsure`` (parents' trials flow to the
    child only), ``break`` (nothing crosses)."""

    NOEFFECT, BREAK, UNSURE = _NOEFFECT, _BREAK, _UNSURE
    types = list(CHANGE_TYPES)
    what = "change"
    _FLOW = {_NOEFFECT: (keep, keep), _UNSURE: (keep, drop), _BREAK: (drop, drop)}

    def __init__(self, change_type):
        self.validate(change_type)
        self.change_type = change_type

    @classmethod
    def validate(cls, change_type):
        if change_type not in CHANGE_TYPES:
            raise ValueError(f"{change_type!r} is not a {cls.what} change type; expected one "
                             f"of {list(CHANGE_TYPES)}")

    def _rules(self):
        return self._FLOW[self.change_type]

    def _fields(self):
        return {"change_type": self.change_type}


class CodeChange(_ChangeKind):
    what = "code"


class CommandLineChange(_ChangeKind):
    what = "command line"


class ScriptConfigChange(_ChangeKind):
    what = "script configuration"


class CompositeAdapter(BaseAdapter):
    """A chain of adapters: forward in order, backward in reverse order."""

    def __init__(self, *adapters):
        bad = [a for a in adapters if not isinstance(a, BaseAdapter)]
        if bad:
            raise TypeError(f"a composite holds adapter objects only, got "
                            f"{[type(a).__name__ for a in bad]}")
        self.adapters = adapters

    def forward(self, trials):
        for a in self.adapters:
            trials = a.forward(trials)
        return trials

    def backward(self, trials):
        for a in reversed(self.adapters):
            trials = a.backward(trials)
        return trials

    def to_dict(self):
        return None

    @property
    def configuration(self):
        confs = [a.configuration for a in self.adapters]
        if len(confs) == 1:
            return confs[0]
        return [c[0] if len(c) == 1 else c for c in confs]


_REGISTRY: Dict[str, type] = {c.__name__.lower(): c for c in (
    CompositeAdapter, DimensionAddition, DimensionDeletion, DimensionPriorChange,
    DimensionRenaming, AlgorithmChange, CodeChange, CommandLineChange, ScriptConfigChange)}


class Adapter:
    """Factory: ``Adapter(of_type="dimensionaddition", param=...)``; ``Adapter.build(list)``."""

    types = _REGISTRY

    def __new__(cls, of_type, **fields):
        try:
            kind = _REGISTRY[str(of_type).lower()]
        except KeyError:
            raise NotImplementedError(f"no BaseAdapter implementation named '{of_type}'; "
                                      f"known: {sorted(_REGISTRY)}") from None
        return kind(**fields)

    @classmethod
    def build(cls, configuration) -> CompositeAdapter:
        members = []
        for entry in configuration or []:
            members.append(cls.build(entry) if isinstance(entry, (list, tuple))
                           else cls(**entry))
        return CompositeAdapter(*members)
