"""Study-level ``suggest()`` / ``observe(trial, results)`` API (reference ROADMAP.md:24-35).

    study = register("fct-dummy", x="loguniform(0.1, 1)")
    trial = study.suggest()
    study.observe(trial, [{"name": "loss", "type": "objective", "value": f(**trial.arguments)}])

Any number of processes may share a study through a file/Mongo database: ``suggest`` uses the
same atomic reserve and duplicate-safe production as the worker loop, and each suggested trial is
kept alive by the heartbeat thread until it is observed (``heartbeat=True``).
"""
from __future__ import annotations

import datetime
import logging
from typing import Dict, List, Optional, Union

from ..core.trial import Trial
from ..worker.pacemaker import TrialPacemaker
from ..worker.producer import Producer
from ..worker.workon import reserve_trial

log = logging.getLogger(__name__)


def _normalize_results(results) -> List[dict]:
    if isinstance(results, (int, float)):
        return [dict(name="objective", type="objective", value=float(results))]
    if isinstance(results, dict):
        if "type" in results:
            return [results]
        out = []
        for i, (k, v) in enumerate(results.items()):
            out.append(dict(name=k, type="objective" if i == 0 else "statistic", value=v))
        return out
    return list(results)


class Study:
    def __init__(self, experiment, heartbeat=False):
        self.experiment = experiment
        self.producer = Producer(experiment)
        self._pacemakers: Dict[str, TrialPacemaker] = {}
        self.heartbeat = heartbeat

    @property
    def space(self):
        return self.experiment.space

    @property
    def is_done(self):
        return self.experiment.is_done

    def suggest(self) -> Optional[Trial]:
        trial = reserve_trial(self.experiment, self.producer)
        if trial is not None and self.heartbeat:
            pm = TrialPacemaker(trial, storage=self.experiment.storage)
            pm.start()
            self._pacemakers[trial.id] = pm
        return trial

    def observe(self, trial: Trial, results: Union[float, dict, list]):
        trial.results = [Trial.Result(**r) for r in _normalize_results(results)]
        trial.status = "completed"
        trial.end_time = datetime.datetime.utcnow()
        self.experiment.storage.push_trial_results(trial)
        pm = self._pacemakers.pop(trial.id, None)
        if pm is not None:
            pm.stop()

    def release(self, trial: Trial, status="interrupted"):
        """Give a suggested trial back (or mark it broken)."""
        self.experiment.set_trial_status(trial, status=status)
        pm = self._pacemakers.pop(trial.id, None)
        if pm is not None:
            pm.stop()

    def fetch_trials(self, with_evc_tree=False):
        return self.experiment.fetch_trials(with_evc_tree=with_evc_tree)

    @property
    def stats(self):
        return self.experiment.stats

    def close(self):
        for pm in self._pacemakers.values():
            pm.stop()
        self._pacemakers.clear()


def register(experiment: str, algorithms="random", max_trials=float("inf"), pool_size=1,
             storage=None, strategy=None, **priors) -> Study:
    """Create or reload the experiment ``experiment`` with priors given as keyword arguments."""
    from ..io.experiment_builder import build_experiment
    from ..storage.protocol import setup_storage, storage_is_set
    if storage is None and not storage_is_set():
        storage = setup_storage(debug=True)
    named = {(k if k.startswith("/") else "/" + k): v for k, v in priors.items()}
    exp = build_experiment(experiment, priors=named, algorithms=algorithms, max_trials=max_trials,
                           pool_size=pool_size, storage=storage, strategy=strategy)
    return Study(exp)
