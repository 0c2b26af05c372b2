"""Consumer: evaluates one trial by running the user's script as a black-box subprocess.

Behaviour contract (reference ``src/orion/core/worker/consumer.py:37-199``): each trial runs in
a working directory ``<working_dir>/<experiment>_<trial id>`` (temporary unless the experiment
sets ``working_dir``) holding the trial's rendered configuration file and the results file the
script writes through ``report_results``; the script sees ``ORION_EXPERIMENT_ID / _NAME /
_VERSION``, ``ORION_TRIAL_ID``, ``ORION_WORKING_DIR`` and ``ORION_RESULTS_PATH`` (plus
``MOPT_*`` twins); the trial's heartbeat is kept while it runs.  Outcome: exit code 0 -> the
results are recorded (``completed``); non-zero -> ``broken``; SIGTERM or Ctrl-C ->
``interrupted`` and the interruption propagates.

Structure: :class:`TrialFiles` lays out one trial's directory and files, :func:`trial_env`
builds its environment, and :meth:`Consumer.consume` maps the run's outcome onto the trial's
status.  The SIGTERM -> KeyboardInterrupt handler is installed once per consumer (not once per
trial, reference quirk 11).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import tempfile
import threading
from dataclasses import dataclass

from ..core.config import config as global_config
from ..io.space_parser import SpaceCmdlineParser
from ..utils.working_dir import WorkingDir
from .pacemaker import TrialPacemaker

log = logging.getLogger(__name__)


class ExecutionError(Exception):
    """The user's script exited with a non-zero code."""


def _raise_interrupt(signum, frame):
    log.error("worker interrupted (SIGTERM)")
    raise KeyboardInterrupt


@dataclass
class TrialFiles:
    """The rendered configuration and the (empty) results file of one trial, in ``root``."""
    root: str
    config: str
    results: str

    @classmethod
    def create(cls, root: str) -> "TrialFiles":
        paths = []
        for prefix, suffix in (("trial_", ".conf"), ("results_", ".log")):
            fd, path = tempfile.mkstemp(prefix=prefix, suffix=suffix, dir=root)
            os.close(fd)
            paths.append(path)
        return cls(root, *paths)


# the directory holding the ``metaopt_amd`` and ``orion`` packages of this worker
_PACKAGE_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _client_importable(env: dict) -> dict:
    """Make the worker's own client library importable by the script (``from orion.client
    import report_results``), as an installed distribution would: the package root is appended
    to ``PYTHONPATH`` unless the packages are already importable from site-packages or the path
    already holds it."""
    import importlib.util
    spec = importlib.util.find_spec("orion")
    installed = spec is not None and spec.origin is not None and "site-packages" in spec.origin
    paths = [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p]
    if not installed and _PACKAGE_ROOT not in paths and \
            os.path.isdir(os.path.join(_PACKAGE_ROOT, "orion")):
        env["PYTHONPATH"] = os.pathsep.join(paths + [_PACKAGE_ROOT])
    return env


def trial_env(experiment, trial, results_path, base=None) -> dict:
    """The script's environment: ``base`` (default: this process's) plus the trial variables
    under both the ``ORION_`` and ``MOPT_`` prefixes, with the client library importable."""
    env = _client_importable(dict(os.environ if base is None else base))
    values = {"EXPERIMENT_ID": experiment.id, "EXPERIMENT_NAME": experiment.name,
              "EXPERIMENT_VERSION": experiment.version, "TRIAL_ID": trial.id,
              "WORKING_DIR": trial.working_dir, "RESULTS_PATH": results_path}
    for prefix in ("ORION", "MOPT"):
        env.update({f"{prefix}_{k}": str(v) for k, v in values.items()})
    return env


class Consumer:
    def __init__(self, experiment, heartbeat=None):
        if experiment.space is None:
            raise RuntimeError("the experiment is not configured yet (no space): the Consumer "
                               "needs a built experiment")
        self.experiment = experiment
        self.space = experiment.space
        self.template_builder = SpaceCmdlineParser(global_config.user_script_config)
        self.template_builder.set_state_dict(experiment.metadata["parser"])
        self.working_dir = (os.path.abspath(experiment.working_dir) if experiment.working_dir
                            else os.path.join(tempfile.gettempdir(), "mopt"))
        self.script_path = experiment.metadata["user_script"]
        self.heartbeat = (global_config.worker.pacemaker_interval if heartbeat is None
                          else heartbeat)
        self.pacemaker = None
        if threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGTERM, _raise_interrupt)

    def consume(self, trial) -> None:
        """Run ``trial`` and record its outcome in the experiment's storage."""
        exp = self.experiment
        try:
            with WorkingDir(self.working_dir, exp.working_dir is None,
                            prefix=exp.name + "_", suffix=trial.id) as wd:
                trial.working_dir = wd
                files = TrialFiles.create(wd)
                self._run(trial, files)
                exp.update_completed_trial(trial, files.results)
        except KeyboardInterrupt:
            exp.set_trial_status(trial, status="interrupted")
            raise
        except (ExecutionError, ValueError) as exc:
            log.warning("trial %s broke: %s", trial.id, exc)
            exp.set_trial_status(trial, status="broken")

    def get_execution_environment(self, trial, results_file="results.log") -> dict:
        return trial_env(self.experiment, trial, results_file)

    def _run(self, trial, files: TrialFiles) -> None:
        args = self.template_builder.format(files.config, trial, self.experiment)
        env = self.get_execution_environment(trial, files.results)
        self.pacemaker = TrialPacemaker(trial, wait_time=self.heartbeat,
                                        storage=getattr(self.experiment, "storage", None))
        self.pacemaker.start()
        try:
            self.execute_process(args, env)
        finally:
            self.pacemaker.stop()

    def command(self, cmd_args) -> list:
        """``[script] + args``; a non-executable ``.py`` script runs under this interpreter."""
        script = self.script_path
        head = [script]
        if script.endswith(".py") and not os.access(script, os.X_OK):
            head = [sys.executable, script]
        return head + list(cmd_args)

    def execute_process(self, cmd_args, environ) -> None:
        proc = subprocess.Popen(self.command(cmd_args), env=environ)
        try:
            code = proc.wait()
        except KeyboardInterrupt:
            proc.terminate()
            try:
                proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                proc.kill()
            raise
        if code != 0:
            raise ExecutionError(f"the script exited with code {code}; see its output")
