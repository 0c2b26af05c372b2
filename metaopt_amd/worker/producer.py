"""Producer: keeps the algorithm up to date and registers new trials
(reference: ``src/orion/core/worker/producer.py:24-174``).

``update()`` fetches the experiment's trials; completed ones not yet observed are fed to the
algorithm and the parallel strategy; in-flight ones get *lies* (registered in ``lying_trials``)
observed by a deep copy of the algorithm (the "naive" algorithm).  ``produce()`` asks the naive
algorithm for ``pool_size`` points, syncs the RNG state back to the real algorithm and registers
the points as trials; duplicates (same md5 ``_id``) back off and retry, and ``max_idle_time``
bounds the whole loop.

Fixed reference quirk 2: ``backoff`` really sleeps (the reference's ``min(0, gauss(1, .2))`` is
never positive); the wait is capped by ``backoff_max`` so tests stay fast.
"""
from __future__ import annotations

import copy
import logging
import random
import time

from ..core.config import config as global_config
from ..storage.database import DuplicateKeyError
from ..utils import format_trials
from ..utils.exceptions import SampleTimeout
from .trials_history import TrialsHistory

log = logging.getLogger(__name__)


class Producer:
    def __init__(self, experiment, max_idle_time=None, backoff_max=1.0):
        self.experiment = experiment
        self.space = experiment.space
        if self.space is None:
            raise RuntimeError("Experiment object provided to Producer has not yet completed"
                               " initialization.")
        self.algorithm = experiment.algorithms
        self.max_idle_time = (global_config.worker.max_idle_time if max_idle_time is None
                              else max_idle_time)
        self.strategy = experiment.producer["strategy"]
        self.naive_algorithm = None
        self.trials_history = TrialsHistory()
        self.naive_trials_history = None
        self.backoff_max = backoff_max

    @property
    def pool_size(self):
        return self.experiment.pool_size

    def backoff(self):
        wait = max(0.0, min(self.backoff_max, random.gauss(self.backoff_max / 2,
                                                           self.backoff_max / 10)))
        log.info("Waiting %.2f seconds", wait)
        time.sleep(wait)
        self.update()

    def produce(self):
        sampled = 0
        start = time.time()
        if self.naive_algorithm is None:
            self.update()
        while sampled < self.pool_size and not self.algorithm.is_done:
            if time.time() - start > self.max_idle_time:
                raise SampleTimeout(f"Algorithm could not sample new points in less than "
                                    f"{self.max_idle_time} seconds")
            new_points = self.naive_algorithm.suggest(self.pool_size - sampled)
            self.algorithm.set_state(self.naive_algorithm.state_dict)
            if new_points is None:
                log.info("### Algo opted out.")
                self.backoff()
                continue
            for point in new_points:
                trial = format_trials.tuple_to_trial(point, self.space)
                try:
                    trial.parents = self.naive_trials_history.children
                    self.experiment.register_trial(trial)
                    sampled += 1
                except DuplicateKeyError:
                    log.debug("#### Duplicate sample.")
                    self.backoff()
                    break
        return sampled

    def update(self):
        trials = self.experiment.fetch_trials()
        self._update_algorithm([t for t in trials if t.status == "completed"])
        self._update_naive_algorithm([t for t in trials if t.status != "completed"])

    def _update_algorithm(self, completed):
        new = [t for t in completed if t not in self.trials_history]
        if not new:
            return
        points = [format_trials.trial_to_tuple(t, self.space) for t in new]
        results = [format_trials.get_trial_results(t) for t in new]
        self.trials_history.update(new)
        self.algorithm.observe(points, results)
        self.strategy.observe(points, results)

    def _produce_lies(self, incomplete):
        lies = []
        for trial in incomplete:
            if trial.status == "broken":
                continue
            result = self.strategy.lie(trial)
            if result is None:
                continue
            lying = copy.deepcopy(trial)
            lying.results.append(result)
            lying.parents = self.trials_history.children
            lies.append(lying)
            try:
                self.experiment.register_lie(lying)
            except DuplicateKeyError:
                log.debug("#### Duplicate lie.")
        return lies

    def _update_naive_algorithm(self, incomplete):
        self.naive_algorithm = copy.deepcopy(self.algorithm)
        self.naive_trials_history = copy.deepcopy(self.trials_history)
        lies = self._produce_lies(incomplete)
        if lies:
            points = [format_trials.trial_to_tuple(t, self.space) for t in lies]
            results = [format_trials.get_trial_results(t) for t in lies]
            self.naive_trials_history.update(lies)
            self.naive_algorithm.observe(points, results)
