"""Manual insertion of trials (reference: ``src/orion/client/manual.py:16-59``)."""
from __future__ import annotations

import logging

from ..storage.database import DuplicateKeyError
from ..utils import format_trials

log = logging.getLogger(__name__)


def insert_trials(experiment_name, points, cmdconfig=None, raise_exc=True, storage=None):
    """Register ``points`` (tuples in the experiment space order) as new trials."""
    from ..io.experiment_builder import ExperimentBuilder
    cmdconfig = dict(cmdconfig or {})
    cmdconfig["name"] = experiment_name
    builder = ExperimentBuilder(storage=storage)
    experiment = builder.build_view_from(cmdconfig)._experiment
    valid = []
    for point in points:
        if point not in experiment.space:
            if raise_exc:
                raise ValueError(f"Point {point} does not belong to the space {experiment.space}")
            log.warning("Point %s is outside the space; skipped", point)
            continue
        valid.append(point)
    new = []
    storage = experiment._storage
    if hasattr(storage, "_storage"):  # a view wraps the writable storage read-only
        storage = storage._storage
    import datetime
    for p in valid:
        t = format_trials.tuple_to_trial(p, experiment.space)
        t.experiment = experiment.id
        t.status = "new"
        t.submit_time = datetime.datetime.utcnow()
        try:
            storage.register_trial(t)
            new.append(t)
        except DuplicateKeyError:
            if raise_exc:
                raise
            log.warning("Point %s already registered", p)
    return new
