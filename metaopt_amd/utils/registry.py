"""Plugin registries (the reference's ``Factory`` metaclass, ``src/orion/core/utils/__init__.py:80-159``).

A :class:`Registry` maps lower-cased names to classes.  Built-in classes register themselves with
``@REGISTRY.register()``; external packages register through ``importlib.metadata`` entry points
(the reference used deprecated ``pkg_resources``).  Each registry reads the entry-point groups it
was created with, e.g. algorithms read ``metaopt_amd.algorithms`` and the reference-compatible
``OptimizationAlgorithm`` group, so an Oríon-style plugin package installs unchanged.
"""
from __future__ import annotations

import importlib
import logging
from importlib import metadata
from typing import Dict, Iterable, Optional, Type

log = logging.getLogger(__name__)


class Registry:
    def __init__(self, kind: str, groups: Iterable[str] = (), builtin_modules: Iterable[str] = ()):
        self.kind = kind
        self.groups = tuple(groups)
        self.builtin_modules = tuple(builtin_modules)
        self._types: Dict[str, type] = {}
        self._loaded = False

    def register(self, name: Optional[str] = None):
        def deco(cls):
            self.add(cls, name)
            return cls
        return deco

    def add(self, cls, name: Optional[str] = None):
        key = (name or cls.__name__).lower()
        self._types[key] = cls
        return cls

    def _load(self):
        if self._loaded:
            return
        self._loaded = True
        for mod in self.builtin_modules:
            try:
                importlib.import_module(mod)
            except Exception as exc:  # pragma: no cover - optional builtins
                log.debug("could not import %s: %s", mod, exc)
        for group in self.groups:
            try:
                eps = metadata.entry_points(group=group)
            except TypeError:  # pragma: no cover - python < 3.10 API
                eps = metadata.entry_points().get(group, [])
            for ep in eps:
                try:
                    self.add(ep.load(), ep.name)
                except Exception as exc:  # pragma: no cover - broken third-party plugin
                    log.warning("could not load %s plugin %s: %s", self.kind, ep.name, exc)

    @property
    def types(self) -> Dict[str, type]:
        self._load()
        return dict(self._types)

    def names(self):
        return sorted(self.types)

    def get(self, of_type: str) -> type:
        self._load()
        key = str(of_type).lower()
        if key not in self._types:
            raise NotImplementedError(
                f"Could not find implementation of {self.kind}, type = '{of_type}'\n"
                f"Currently, there is an implementation for types:\n{sorted(self._types)}")
        return self._types[key]

    def __call__(self, of_type: str, *args, **kwargs):
        return self.get(of_type)(*args, **kwargs)

    def __contains__(self, of_type):
        self._load()
        return str(of_type).lower() in self._types
