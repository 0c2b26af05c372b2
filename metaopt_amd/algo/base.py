"""Algorithm interface and registry (reference: ``src/orion/algo/base.py:21-279``).

An algorithm proposes points of a :class:`~metaopt_amd.space.dims.Space` with
``suggest(num)`` and learns from evaluations with ``observe(points, results)`` where each result
is ``{'objective': float|None, 'constraint': [...], 'gradient': tuple|None}``.

Keyword arguments given to ``BaseAlgorithm.__init__`` are the algorithm's tunable parameters and
make up its ``configuration`` (``{name_lower: {param: value}}``), which experiments persist.  A
kwarg that names another registered algorithm (a string, or ``{name: {kwargs}}``) is
instantiated as a nested algorithm on the same space; ``seed`` calls :meth:`seed_rng`.

Registry: ``ALGORITHMS`` (entry-point groups ``metaopt_amd.algorithms`` and the reference's
``OptimizationAlgorithm``), so Oríon-style plugin packages register unchanged.
"""
from __future__ import annotations

import copy
import logging
from typing import List, Optional

from ..utils.registry import Registry

log = logging.getLogger(__name__)

ALGORITHMS = Registry("OptimizationAlgorithm",
                      groups=("metaopt_amd.algorithms", "OptimizationAlgorithm"),
                      builtin_modules=("metaopt_amd.algo.random", "metaopt_amd.algo.asha",
                                       "metaopt_amd.algo.tpe", "metaopt_amd.algo.gridsearch",
                                       "metaopt_amd.algo.pbt", "metaopt_amd.algo.hyperband",
                                       "metaopt_amd.algo.gradient_descent"))


class BaseAlgorithm:
    """Base class of every search algorithm.

    ``requires`` names the space type the algorithm needs (None, 'real' or 'integer'); the
    experiment wraps it in :class:`~metaopt_amd.algo.primary.PrimaryAlgo`, which transforms the
    space accordingly.
    """

    requires: Optional[str] = None
    #: True when suggestions at a sync depend on the results of trials finishing at that same
    #: sync (PBT generations); device sweeps then decide synchronously instead of one interval
    #: behind the GPU (see ``PopulationSweep``)
    synchronous: bool = False
    #: True for built-in algorithms whose points are draws of ``space.sample`` (or earlier
    #: points): the primary wrapper then skips re-validating every suggested point
    trusted_suggestions: bool = False

    def __init__(self, space, **kwargs):
        log.debug("Creating %s with parameters %s", type(self).__name__, kwargs)
        self._space = space
        self._param_names = list(kwargs.keys())
        for varname, param in kwargs.items():
            if isinstance(param, dict) and len(param) == 1 and \
                    isinstance(next(iter(param.values())), dict) and next(iter(param)) in ALGORITHMS:
                sub_type = next(iter(param))
                param = ALGORITHMS(sub_type, space, **param[sub_type])
            elif isinstance(param, str) and param.lower() in ALGORITHMS and varname != "seed":
                param = ALGORITHMS(param, space)
            elif varname == "seed":
                self.seed_rng(param)
            setattr(self, varname, param)

    def seed_rng(self, seed):
        """Seed the algorithm's RNG (no-op for deterministic algorithms)."""

    @property
    def state_dict(self) -> dict:
        """State that ``set_state`` restores (the RNG for sampling algorithms)."""
        return {}

    def set_state(self, state_dict: dict) -> None:
        pass

    def full_state(self) -> dict:
        """Everything ``set_state`` needs to continue the search itself (observations, rungs,
        lineage) -- persisted with an experiment; ``state_dict`` may be the RNG alone (the
        producer syncs only the RNG between its naive and real algorithm copies)."""
        return self.state_dict

    def suggest(self, num=1) -> Optional[List[tuple]]:
        """Up to ``num`` new points, or None to opt out (e.g. waiting for running trials)."""
        raise NotImplementedError

    def observe(self, points, results) -> None:
        raise NotImplementedError

    @property
    def is_done(self) -> bool:
        return False

    def score(self, point) -> float:
        return 0

    def judge(self, point, measurements):
        return None

    @property
    def should_suspend(self) -> bool:
        return False

    @property
    def space(self):
        return self._space

    @space.setter
    def space(self, space):
        self._space = space

    @property
    def configuration(self) -> dict:
        params = {}
        for name in self._param_names:
            attr = getattr(self, name)
            if isinstance(attr, BaseAlgorithm):
                attr = attr.configuration
            params[name] = attr
        return {type(self).__name__.lower(): params}

    def clone(self):
        return copy.deepcopy(self)


def create_algo(space, config) -> BaseAlgorithm:
    """``create_algo(space, 'random')`` or ``create_algo(space, {'asha': {'seed': 1}})``."""
    if isinstance(config, str):
        return ALGORITHMS(config, space)
    if isinstance(config, dict) and len(config) == 1:
        name, kwargs = next(iter(config.items()))
        return ALGORITHMS(name, space, **(kwargs or {}))
    raise ValueError(f"Invalid algorithm configuration: {config!r}")
