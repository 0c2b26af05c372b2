"""Parallel strategies: fake objectives ("lies") for trials still in flight so sequential
algorithms can be used by many asynchronous workers
(reference: ``src/orion/core/worker/strategy.py:20-158``).

* ``NoParallelStrategy``   -- no lie (the pending trial is ignored)
* ``MaxParallelStrategy``  -- lie with the worst (max) objective observed so far (default;
  the reference documents "best" but implements max, quirk 3 -- max is kept: it is the
  conservative choice that pushes the algorithm away from pending points)
* ``MeanParallelStrategy`` -- lie with the mean observed objective
* ``StubParallelStrategy`` -- lie with a fixed ``stub_value``
"""
from __future__ import annotations

import logging

from ..core.trial import Trial
from ..utils.registry import Registry

log = logging.getLogger(__name__)

STRATEGIES = Registry("ParallelStrategy", groups=("metaopt_amd.strategies",))


def get_objective(trial):
    obj = trial.objective
    return obj.value if obj is not None else None


class BaseParallelStrategy:
    def observe(self, points, results):
        raise NotImplementedError

    def lie(self, trial):
        if get_objective(trial) is not None:
            raise RuntimeError("Trial {} is completed but should not be.".format(trial.id))

    @property
    def configuration(self):
        return self.__class__.__name__


@STRATEGIES.register()
class NoParallelStrategy(BaseParallelStrategy):
    def observe(self, points, results):
        pass

    def lie(self, trial):
        super().lie(trial)
        return None


@STRATEGIES.register()
class MaxParallelStrategy(BaseParallelStrategy):
    def __init__(self, default_result=float("inf")):
        self.default_result = default_result
        self.max_result = None

    def observe(self, points, results):
        objs = [r["objective"] for r in results if r.get("objective") is not None]
        if objs:
            m = max(objs)
            self.max_result = m if self.max_result is None else max(self.max_result, m)

    def lie(self, trial):
        super().lie(trial)
        val = self.max_result if self.max_result is not None else self.default_result
        return Trial.Result(name="lie", type="lie", value=val)


@STRATEGIES.register()
class MeanParallelStrategy(BaseParallelStrategy):
    def __init__(self, default_result=float("inf")):
        self.default_result = default_result
        self._sum = 0.0
        self._n = 0

    def observe(self, points, results):
        objs = [r["objective"] for r in results if r.get("objective") is not None]
        self._sum += sum(objs)
        self._n += len(objs)

    @property
    def mean_result(self):
        return self._sum / self._n if self._n else None

    def lie(self, trial):
        super().lie(trial)
        val = self.mean_result if self._n else self.default_result
        return Trial.Result(name="lie", type="lie", value=val)


@STRATEGIES.register()
class StubParallelStrategy(BaseParallelStrategy):
    def __init__(self, stub_value=None):
        self.stub_value = stub_value

    def observe(self, points, results):
        pass

    def lie(self, trial):
        super().lie(trial)
        return Trial.Result(name="lie", type="lie", value=self.stub_value)

    @property
    def configuration(self):
        return {"StubParallelStrategy": {"stub_value": self.stub_value}}


def create_strategy(config=None) -> BaseParallelStrategy:
    """``'MaxParallelStrategy'`` or ``{'StubParallelStrategy': {'stub_value': 1}}``."""
    if config is None:
        return MaxParallelStrategy()
    if isinstance(config, str):
        return STRATEGIES(config)
    if isinstance(config, dict) and len(config) == 1:
        name, kwargs = next(iter(config.items()))
        return STRATEGIES(name, **(kwargs or {}))
    raise ValueError(f"Invalid strategy configuration {config!r}")
