"""Adapters carry trials across a branch of the experiment version-control tree
(reference: ``src/orion/core/evc/adapters.py:45-869``).

``forward(parent_trials)`` makes a parent's trials valid for the child, ``backward(child_trials)``
makes a child's trials valid for the parent.  Every adapter serialises with ``to_dict`` (stored in
the child's ``refers.adapter`` as a list of dicts) and is rebuilt with :meth:`Adapter.build`.

=====================  ==========================================  =============================
adapter                forward (parent -> child)                   backward (child -> parent)
=====================  ==========================================  =============================
DimensionAddition      add the param with its default value        keep trials at the default,
                                                                   drop the param
DimensionDeletion      keep trials at the default, drop the param  add the param (default)
DimensionPriorChange   keep trials inside the new prior            keep trials inside the old
DimensionRenaming      rename old -> new                           rename new -> old
AlgorithmChange        pass                                        pass
Code/CommandLine/      pass unless ``break``                       pass only for ``noeffect``
ScriptConfig change
CompositeAdapter       apply in order                              apply in reverse order
=====================  ==========================================  =============================
"""
from __future__ import annotations

import copy
from typing import List

from ..core.trial import Param, Trial
from ..space.builder import DimensionBuilder


def apply_if_valid(name, trial, callback=None, raise_if_not=True):
    for param in trial.params:
        if param.name == name:
            return callback is None or callback(trial, param)
    if raise_if_not:
        raise RuntimeError("Provided trial does not have a compatible configuration. "
                           f"A dimension named '{name}' should be present.\n {trial}")
    return False


class BaseAdapter:
    def forward(self, trials: List[Trial]) -> List[Trial]:
        raise NotImplementedError

    def backward(self, trials: List[Trial]) -> List[Trial]:
        raise NotImplementedError

    def to_dict(self) -> dict:
        raise NotImplementedError

    @property
    def configuration(self) -> list:
        return [self.to_dict()]

    def __eq__(self, other):
        return isinstance(other, BaseAdapter) and self.configuration == other.configuration


class CompositeAdapter(BaseAdapter):
    def __init__(self, *adapters):
        for a in adapters:
            if not isinstance(a, BaseAdapter):
                raise TypeError(f"Provided adapters must be adapter objects, not '{type(a)}'")
        self.adapters = adapters

    def forward(self, trials):
        for a in self.adapters:
            trials = a.forward(trials)
        return trials

    def backward(self, trials):
        for a in self.adapters[::-1]:
            trials = a.backward(trials)
        return trials

    def to_dict(self):
        return None

    @property
    def configuration(self):
        if len(self.adapters) > 1:
            return [a.configuration if len(a.configuration) > 1 else a.configuration[0]
                    for a in self.adapters]
        if self.adapters:
            return self.adapters[0].configuration
        return []


def _as_param(param):
    if isinstance(param, dict):
        return Param(**param)
    if isinstance(param, Param):
        return param
    raise TypeError(f"Invalid param argument type ('{type(param)}'). Param argument must be a "
                    "Param object or a dictionnary as defined by Trial.Param.to_dict().")


class DimensionAddition(BaseAdapter):
    def __init__(self, param):
        self.param = _as_param(param)

    def forward(self, trials):
        out = []
        for t in trials:
            if apply_if_valid(self.param.name, t, raise_if_not=False):
                raise RuntimeError("Provided trial does not have a compatible configuration. A "
                                   f"dimension named '{self.param.name}' was already present.\n{t}")
            nt = copy.deepcopy(t)
            nt.params.append(copy.deepcopy(self.param))
            nt.params.sort(key=lambda p: p.name)
            out.append(nt)
        return out

    def backward(self, trials):
        out = []

        def keep_default(trial, param):
            if param.value == self.param.value:
                nt = copy.deepcopy(trial)
                nt.params = [p for p in nt.params if p.name != self.param.name]
                out.append(nt)
                return True
            return False

        for t in trials:
            apply_if_valid(self.param.name, t, keep_default, raise_if_not=True)
        return out

    def to_dict(self):
        return dict(of_type="dimensionaddition", param=self.param.to_dict())


class DimensionDeletion(BaseAdapter):
    def __init__(self, param):
        self.dimension_addition_adapter = DimensionAddition(param)

    @property
    def param(self):
        return self.dimension_addition_adapter.param

    def forward(self, trials):
        return self.dimension_addition_adapter.backward(trials)

    def backward(self, trials):
        return self.dimension_addition_adapter.forward(trials)

    def to_dict(self):
        d = self.dimension_addition_adapter.to_dict()
        d["of_type"] = "dimensiondeletion"
        return d


class DimensionPriorChange(BaseAdapter):
    def __init__(self, name, old_prior, new_prior):
        self.name, self.old_prior, self.new_prior = name, old_prior, new_prior
        self.old_dimension = DimensionBuilder().build("old", old_prior)
        self.new_dimension = DimensionBuilder().build("new", new_prior)
        if self.old_dimension.shape != self.new_dimension.shape:
            raise NotImplementedError("Adaptations on prior shape changes are not supported.")

    def forward(self, trials):
        return [t for t in trials
                if apply_if_valid(self.name, t, lambda tr, p: p.value in self.new_dimension)]

    def backward(self, trials):
        return DimensionPriorChange(self.name, self.new_prior, self.old_prior).forward(trials)

    def to_dict(self):
        return dict(of_type="dimensionpriorchange", name=self.name, old_prior=self.old_prior,
                    new_prior=self.new_prior)


class DimensionRenaming(BaseAdapter):
    def __init__(self, old_name, new_name):
        for n in (old_name, new_name):
            if not isinstance(n, str):
                raise TypeError(f"Invalid name type '{type(n)}'. Names must be strings.")
        self.old_name, self.new_name = old_name, new_name

    def forward(self, trials):
        out = copy.deepcopy(trials)

        def rename(trial, param):
            param.name = self.new_name
            return True

        for t in out:
            apply_if_valid(self.old_name, t, rename, raise_if_not=True)
            t.params.sort(key=lambda p: p.name)
        return out

    def backward(self, trials):
        return DimensionRenaming(self.new_name, self.old_name).forward(trials)

    def to_dict(self):
        return dict(of_type="dimensionrenaming", old_name=self.old_name, new_name=self.new_name)


class AlgorithmChange(BaseAdapter):
    def forward(self, trials):
        return trials

    def backward(self, trials):
        return trials

    def to_dict(self):
        return dict(of_type="algorithmchange")


class _ChangeTypeAdapter(BaseAdapter):
    NOEFFECT, BREAK, UNSURE = "noeffect", "break", "unsure"
    types = [NOEFFECT, BREAK, UNSURE]
    kind = "change"

    def __init__(self, change_type):
        self.validate(change_type)
        self.change_type = change_type

    @classmethod
    def validate(cls, change_type):
        if change_type not in cls.types:
            raise ValueError(f"Invalid {cls.kind} change type '{change_type}'. Should be one of "
                             f"{cls.types}")

    def forward(self, trials):
        return [] if self.change_type == self.BREAK else trials

    def backward(self, trials):
        return [] if self.change_type in (self.BREAK, self.UNSURE) else trials

    def to_dict(self):
        return dict(of_type=type(self).__name__.lower(), change_type=self.change_type)


class CodeChange(_ChangeTypeAdapter):
    kind = "code"


class CommandLineChange(_ChangeTypeAdapter):
    kind = "command line"


class ScriptConfigChange(_ChangeTypeAdapter):
    kind = "script configuration"


_TYPES = {c.__name__.lower(): c for c in (CompositeAdapter, DimensionAddition, DimensionDeletion,
                                          DimensionPriorChange, DimensionRenaming, AlgorithmChange,
                                          CodeChange, CommandLineChange, ScriptConfigChange)}


class Adapter:
    """Factory: ``Adapter(of_type='dimensionaddition', param=...)`` / ``Adapter.build([...])``."""

    types = _TYPES

    def __new__(cls, of_type, **kwargs):
        key = str(of_type).lower()
        if key not in _TYPES:
            raise NotImplementedError(f"Could not find implementation of BaseAdapter, "
                                      f"type = '{of_type}'")
        return _TYPES[key](**kwargs)

    @classmethod
    def build(cls, adapter_dicts) -> CompositeAdapter:
        adapters = []
        for d in adapter_dicts or []:
            if isinstance(d, (list, tuple)):
                adapters.append(cls.build(d))
            else:
                adapters.append(cls(**d))
        return CompositeAdapter(*adapters)
