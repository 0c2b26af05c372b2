"""Consumer: evaluates one trial by running the user's script as a subprocess
(reference: ``src/orion/core/worker/consumer.py:37-199``).

Per trial: a working directory ``<working_dir>/<exp>_<trial.id>`` (temporary unless the
experiment sets ``working_dir``), a rendered config file and a results file, environment variables
``ORION_EXPERIMENT_ID/_NAME/_VERSION``, ``ORION_TRIAL_ID``, ``ORION_WORKING_DIR``,
``ORION_RESULTS_PATH`` (plus ``MOPT_*`` aliases), the heartbeat thread, then
``Popen([script] + args)``.  Exit code != 0 -> ``broken``; SIGTERM or Ctrl-C -> ``interrupted``
(re-raised).  The SIGTERM handler is installed once per consumer (reference quirk 11).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import tempfile
import threading

from ..core.config import config as global_config
from ..io.space_parser import SpaceCmdlineParser
from ..utils.working_dir import WorkingDir
from .pacemaker import TrialPacemaker

log = logging.getLogger(__name__)


class ExecutionError(Exception):
    pass


def _sigterm_handler(signum, frame):
    log.error("The worker has been interrupted (SIGTERM).")
    raise KeyboardInterrupt


class Consumer:
    def __init__(self, experiment, heartbeat=None):
        self.experiment = experiment
        self.space = experiment.space
        if self.space is None:
            raise RuntimeError("Experiment object provided to Consumer has not yet completed"
                               " initialization.")
        self.template_builder = SpaceCmdlineParser(global_config.user_script_config)
        self.template_builder.set_state_dict(experiment.metadata["parser"])
        if experiment.working_dir:
            self.working_dir = os.path.abspath(experiment.working_dir)
        else:
            self.working_dir = os.path.join(tempfile.gettempdir(), "mopt")
        self.script_path = experiment.metadata["user_script"]
        self.pacemaker = None
        self.heartbeat = (global_config.worker.pacemaker_interval if heartbeat is None
                          else heartbeat)
        if threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGTERM, _sigterm_handler)

    def consume(self, trial):
        temp = self.experiment.working_dir is None
        try:
            with WorkingDir(self.working_dir, temp, prefix=self.experiment.name + "_",
                            suffix=trial.id) as wd:
                trial.working_dir = wd
                results_file = self._consume(trial, wd)
                self.experiment.update_completed_trial(trial, results_file)
        except KeyboardInterrupt:
            self.experiment.set_trial_status(trial, status="interrupted")
            raise
        except (ExecutionError, ValueError) as exc:
            log.warning("Trial %s broke: %s", trial.id, exc)
            self.experiment.set_trial_status(trial, status="broken")

    def get_execution_environment(self, trial, results_file="results.log"):
        env = dict(os.environ)
        for prefix in ("ORION", "MOPT"):
            env[f"{prefix}_EXPERIMENT_ID"] = str(self.experiment.id)
            env[f"{prefix}_EXPERIMENT_NAME"] = str(self.experiment.name)
            env[f"{prefix}_EXPERIMENT_VERSION"] = str(self.experiment.version)
            env[f"{prefix}_TRIAL_ID"] = str(trial.id)
            env[f"{prefix}_WORKING_DIR"] = str(trial.working_dir)
            env[f"{prefix}_RESULTS_PATH"] = str(results_file)
        return env

    def _consume(self, trial, wd):
        cfg = tempfile.NamedTemporaryFile(mode="w", prefix="trial_", suffix=".conf", dir=wd,
                                          delete=False)
        cfg.close()
        res = tempfile.NamedTemporaryFile(mode="w", prefix="results_", suffix=".log", dir=wd,
                                          delete=False)
        res.close()
        env = self.get_execution_environment(trial, res.name)
        args = self.template_builder.format(cfg.name, trial, self.experiment)
        self.pacemaker = TrialPacemaker(trial, wait_time=self.heartbeat,
                                        storage=getattr(self.experiment, "storage", None))
        self.pacemaker.start()
        try:
            self.execute_process(args, env)
        finally:
            self.pacemaker.stop()
        return res.name

    def execute_process(self, cmd_args, environ):
        command = [self.script_path] + list(cmd_args)
        if not os.access(self.script_path, os.X_OK) and self.script_path.endswith(".py"):
            import sys
            command = [sys.executable] + command
        process = subprocess.Popen(command, env=environ)
        try:
            rc = process.wait()
        except KeyboardInterrupt:
            process.terminate()
            try:
                process.wait(timeout=10)
            except subprocess.TimeoutExpired:
                process.kill()
            raise
        if rc != 0:
            raise ExecutionError(f"Something went wrong. Check logs. Process returned with code "
                                 f"{rc} !")
