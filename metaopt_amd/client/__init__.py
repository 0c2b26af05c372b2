"""User-side API.

* :func:`report_results` -- what a black-box script calls once at the end (reference
  ``src/orion/client/__init__.py:13-48``): writes ``[{name, type, value}]`` as JSON to
  ``$ORION_RESULTS_PATH`` (or ``$MOPT_RESULTS_PATH``); outside a worker it just prints.
* :func:`insert_trials` -- register user-chosen points (``client/manual.py``).
* :func:`register` / :class:`Study` -- the study-level ``suggest()``/``observe(trial, results)``
  API sketched in the reference ROADMAP (v0.2), not implemented there.
"""
from __future__ import annotations

import json
import os

from .manual import insert_trials  # noqa: F401
from .study import Study, register  # noqa: F401

RESULTS_FILENAME = os.getenv("ORION_RESULTS_PATH", os.getenv("MOPT_RESULTS_PATH", None))
if RESULTS_FILENAME and not os.path.isfile(RESULTS_FILENAME):
    raise RuntimeError(f"Results file path provided in environment does not exist: "
                       f"{RESULTS_FILENAME}")
IS_ORION_ON = bool(RESULTS_FILENAME)
_HAS_REPORTED_RESULTS = False


def report_results(data):
    """Report the evaluation of a trial. May be called only once per process."""
    global _HAS_REPORTED_RESULTS
    if _HAS_REPORTED_RESULTS:
        raise RuntimeWarning("Has already reported evaluation results once.")
    path = os.getenv("ORION_RESULTS_PATH", os.getenv("MOPT_RESULTS_PATH", RESULTS_FILENAME))
    if path:
        with open(path, "w") as f:
            json.dump(data, f)
    else:
        print(data)
    _HAS_REPORTED_RESULTS = True
