"""Producer: feeds finished trials to the algorithm and turns its suggestions into trials.

Behaviour contract (reference ``src/orion/core/worker/producer.py:24-174``):

* ``update()`` -- completed trials the algorithm has not seen yet are observed by it and by the
  parallel strategy; every trial still in flight gets a *lie* from the strategy (recorded in the
  ``lying_trials`` collection) which only a scratch copy of the algorithm (the *naive*
  algorithm) observes, so in-flight points are not suggested again;
* ``produce()`` -- the naive algorithm is asked for the missing part of ``pool_size``, its RNG
  state is handed back to the real algorithm, and the points are registered as ``new`` trials
  (lineage: the history's frontier); a duplicate id or an algorithm that opts out waits,
  refreshes and retries, within ``max_idle_time``.

Structure: one pass over the experiment's trials splits them into *fresh results* and *in
flight* (:meth:`_partition`); the naive algorithm is rebuilt from the real one on every
``update``; registration stops at the first duplicate (the rest of that batch is stale) and the
wait before retrying is a real, bounded pause (the reference's ``min(0, gauss(1, 0.2))`` never
sleeps, quirk 2).
"""
from __future__ import annotations

import copy
import logging
import random
import time
from typing import List, Tuple

from ..core.config import config as global_config
from ..storage.database import DuplicateKeyError
from ..utils import format_trials
from ..utils.exceptions import SampleTimeout
from .trials_history import TrialsHistory

log = logging.getLogger(__name__)


class Producer:
    def __init__(self, experiment, max_idle_time=None, backoff_max=1.0):
        if experiment.space is None:
            raise RuntimeError("the experiment is not configured yet (no space): the Producer "
                               "needs a built experiment")
        self.experiment = experiment
        self.space = experiment.space
        self.algorithm = experiment.algorithms
        self.strategy = experiment.producer["strategy"]
        self.max_idle_time = (global_config.worker.max_idle_time if max_idle_time is None
                              else max_idle_time)
        self.backoff_max = backoff_max
        self.trials_history = TrialsHistory()
        self.naive_algorithm = None
        self.naive_trials_history = None

    @property
    def pool_size(self) -> int:
        return self.experiment.pool_size

    # -- observing ------------------------------------------------------------------------------
    def update(self) -> None:
        fresh, in_flight = self._partition(self.experiment.fetch_trials())
        if fresh:
            self._observe(self.algorithm, self.trials_history, fresh, also=self.strategy)
        self.naive_algorithm = copy.deepcopy(self.algorithm)
        self.naive_trials_history = copy.deepcopy(self.trials_history)
        lies = [lie for lie in map(self._lie_for, in_flight) if lie is not None]
        if lies:
            self._observe(self.naive_algorithm, self.naive_trials_history, lies)

    def _partition(self, trials) -> Tuple[list, list]:
        """(completed trials not observed yet, trials still in flight -- broken excluded)."""
        fresh, in_flight = [], []
        for t in trials:
            if t.status == "completed":
                if t not in self.trials_history:
                    fresh.append(t)
            elif t.status != "broken":
                in_flight.append(t)
        return fresh, in_flight

    def _observe(self, algorithm, history, trials, also=None) -> None:
        points = [format_trials.trial_to_tuple(t, self.space) for t in trials]
        results = [format_trials.get_trial_results(t) for t in trials]
        history.update(trials)
        algorithm.observe(points, results)
        if also is not None:
            also.observe(points, results)

    def _lie_for(self, trial):
        """The strategy's fake result for an in-flight trial, recorded as a lying trial."""
        result = self.strategy.lie(trial)
        if result is None:
            return None
        lying = copy.deepcopy(trial)
        lying.results.append(result)
        lying.parents = self.trials_history.children
        try:
            self.experiment.register_lie(lying)
        except DuplicateKeyError:
            log.debug("lie of %s already recorded", trial.id)
        return lying

    # -- producing ------------------------------------------------------------------------------
    def produce(self) -> int:
        """Register up to ``pool_size`` new trials; returns how many were registered."""
        if self.naive_algorithm is None:
            self.update()
        deadline = time.time() + self.max_idle_time
        registered = 0
        while registered < self.pool_size and not self.algorithm.is_done:
            if time.time() > deadline:
                raise SampleTimeout(f"Algorithm could not sample new points in less than "
                                    f"{self.max_idle_time} seconds")
            points = self.naive_algorithm.suggest(self.pool_size - registered)
            self.algorithm.set_state(self.naive_algorithm.state_dict)
            if points is None:
                log.info("the algorithm opted out; waiting for results")
                self.backoff()
                continue
            n, duplicate = self._register(points)
            registered += n
            if duplicate:
                self.backoff()
        return registered

    def _register(self, points) -> Tuple[int, bool]:
        """Register ``points`` in order; stops at the first one already stored (True)."""
        n = 0
        for point in points:
            trial = format_trials.tuple_to_trial(point, self.space)
            trial.parents = self.naive_trials_history.children
            try:
                self.experiment.register_trial(trial)
            except DuplicateKeyError:
                log.debug("point %s already registered", point)
                return n, True
            n += 1
        return n, False

    def backoff(self) -> None:
        """Pause (about half of ``backoff_max``, jittered) and refresh the algorithms."""
        wait = max(0.0, min(self.backoff_max,
                            random.gauss(self.backoff_max / 2, self.backoff_max / 10)))
        log.info("waiting %.2f s before sampling again", wait)
        time.sleep(wait)
        self.update()
