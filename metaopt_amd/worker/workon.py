"""The worker loop (reference: ``src/orion/core/worker/__init__.py:24-88``).

Each iteration: stop if ``is_broken`` (>= ``worker.max_broken`` broken trials) or ``is_done``;
reserve a trial (sweeping lost trials first); if none is reservable, update the algorithm,
produce ``pool_size`` new trials and retry -- iteratively, with a bound (the reference recurses
without one, quirk 10); then consume.  Prints RESULTS and BEST PARAMETERS at the end.
"""
from __future__ import annotations

import io
import itertools
import logging
import pprint
import time

from .consumer import Consumer
from .producer import Producer

log = logging.getLogger(__name__)


def reserve_trial(experiment, producer, max_attempts=100, wait=0.1):
    for _ in range(max_attempts):
        trial = experiment.reserve_trial()
        if trial is not None or experiment.is_done:
            return trial
        producer.update()
        produced = producer.produce()
        if not produced:
            time.sleep(wait)  # other workers hold the remaining trials
    return None


def workon(experiment, worker_trials=None, consumer=None, producer=None):
    """Run trials of ``experiment`` until it is done/broken or ``worker_trials`` are consumed."""
    producer = producer or Producer(experiment)
    consumer = consumer or Consumer(experiment)
    try:
        iterator = range(int(worker_trials))
    except (OverflowError, TypeError, ValueError):
        iterator = itertools.count()
    for _ in iterator:
        if experiment.is_broken:
            log.info("#### Experiment has reached broken trials threshold, terminating.")
            return experiment.stats
        if experiment.is_done:
            break
        trial = reserve_trial(experiment, producer)
        if trial is not None:
            consumer.consume(trial)
    return report(experiment)


def report(experiment):
    stats = experiment.stats
    if not stats:
        log.info("No trials completed.")
        return stats
    best = experiment.get_trial(uid=stats["best_trials_id"])
    s = io.StringIO()
    pprint.pprint(stats, stream=s)
    b = io.StringIO()
    pprint.pprint(best.to_dict()["params"], stream=b)
    log.info("#####  Search finished successfully  #####")
    log.info("\nRESULTS\n=======\n%s\n", s.getvalue())
    log.info("\nBEST PARAMETERS\n===============\n%s", b.getvalue())
    return stats
