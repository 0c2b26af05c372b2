"""Build experiments from command-line arguments and configuration files
(reference: ``src/orion/core/io/experiment_builder.py:105-308`` and ``core/io/evc_builder.py``).

``fetch_full_config`` merges, lowest to highest precedence: defaults < env vars < the stored
experiment < the ``--config`` file < command-line arguments < metadata.  ``build_from`` creates or
loads the experiment, parses the user command line into ``metadata.parser`` / ``metadata.priors``,
calls ``Experiment.configure`` (branching through the EVC as needed) and connects the experiment
to its version-control tree; a race on the ``(name, version)`` index is retried once (and, unlike
the reference -- quirk 1 -- a successful retry is returned instead of re-raised).
"""
from __future__ import annotations

import copy
import logging

from ..core.config import config as global_config
from ..core.experiment import Experiment, ExperimentView
from ..evc.experiment_node import ExperimentNode
from ..storage.database import DuplicateKeyError
from ..storage.protocol import get_storage, setup_storage, storage_is_set
from ..utils.exceptions import NoConfigurationError, RaceCondition
from . import resolve_config
from .space_parser import SpaceCmdlineParser

log = logging.getLogger(__name__)

BRANCHING_KEYS = ("branch", "manual_resolution", "auto_resolution", "algorithm_change",
                  "code_change_type", "cli_change_type", "config_change_type")


class ExperimentBuilder:
    def __init__(self, storage=None):
        self._storage = storage

    # -- configuration sources ----------------------------------------------------------------
    def fetch_default_options(self):
        return resolve_config.fetch_default_options()

    def fetch_env_vars(self):
        return resolve_config.fetch_env_vars()

    def fetch_file_config(self, cmdargs):
        return resolve_config.fetch_config(cmdargs)

    def fetch_metadata(self, cmdargs):
        return resolve_config.fetch_metadata(cmdargs)

    def fetch_config_from_db(self, cmdargs):
        try:
            view = self.build_view_from(cmdargs)
        except ValueError as exc:
            if "No experiment with given name" in str(exc):
                return {}
            raise
        return view.configuration

    def fetch_full_config(self, cmdargs, use_db=True):
        cmdargs = {k: v for k, v in dict(cmdargs).items()}
        defaults = self.fetch_default_options()
        env = self.fetch_env_vars()
        from_db = self.fetch_config_from_db(cmdargs) if use_db else {}
        file_cfg = self.fetch_file_config(cmdargs)
        metadata = dict(metadata=self.fetch_metadata(cmdargs))
        cmd = {k: v for k, v in cmdargs.items() if k not in ("config", "user_args")}
        exp_config = resolve_config.merge_configs(defaults, env, copy.deepcopy(from_db), file_cfg,
                                                  cmd, metadata)
        if "user" in exp_config:
            exp_config["metadata"]["user"] = exp_config["user"]
        if isinstance(exp_config.get("algorithms"), dict) and len(exp_config["algorithms"]) > 1 \
                and from_db.get("algorithms"):
            for key in list(from_db["algorithms"].keys()):
                exp_config["algorithms"].pop(key, None)
        return exp_config

    # -- storage ------------------------------------------------------------------------------
    def setup_storage(self, config):
        if self._storage is not None:
            return self._storage
        if storage_is_set() and not config.get("force_storage"):
            return get_storage()  # process-wide storage: the first configuration wins
        db = dict(config.get("database") or {})
        return setup_storage({"database": db}, debug=bool(config.get("debug")))

    # -- builders -----------------------------------------------------------------------------
    def build_view_from(self, cmdargs):
        local = self.fetch_full_config(cmdargs, use_db=False)
        storage = self.setup_storage(local)
        if local.get("name") is None:
            raise RuntimeError("Could not infer experiment's name. Please use either `name` cmd "
                               "line arg or provide one in the configuration file.")
        view = ExperimentView(local["name"], user=local.get("user"), version=local.get("version"),
                              storage=storage)
        self._connect(view)
        return view

    def build_from(self, cmdargs, handle_racecondition=True):
        full = self.fetch_full_config(cmdargs)
        try:
            return self.build_from_config(full)
        except (DuplicateKeyError, RaceCondition):
            if handle_racecondition:
                return self.build_from(cmdargs, handle_racecondition=False)
            raise

    def build_from_config(self, config):
        config = copy.deepcopy(config)
        storage = self.setup_storage(config)
        config.pop("database", None)
        config.pop("resources", None)
        config.pop("debug", None)
        config["branching"] = {k: config.pop(k) for k in BRANCHING_KEYS if k in config}
        experiment = Experiment(config["name"], config.get("user"), config.get("version"),
                                storage=storage)
        md = config.setdefault("metadata", {})
        if "priors" not in md and "user_args" not in md:
            raise NoConfigurationError(f"No configuration for experiment '{config['name']}'")
        if "user_args" in md:
            parser = SpaceCmdlineParser(global_config.user_script_config)
            parser.parse(md["user_args"])
            md["parser"] = parser.get_state_dict()
            md["priors"] = dict(parser.priors)
        # branching flags are also looked up at the top level by conflict resolutions
        for k, v in config["branching"].items():
            if v is not None:
                config[k] = v
        experiment.configure(config)
        for k in BRANCHING_KEYS:
            config.pop(k, None)
        self._connect(experiment)
        return experiment

    @staticmethod
    def _connect(experiment):
        node = ExperimentNode(experiment.name, experiment.version, experiment=experiment,
                              storage=experiment.storage if hasattr(experiment, "storage")
                              else None)
        experiment.connect_to_version_control_tree(node)
        return experiment


# The reference splits these into ExperimentBuilder and EVCBuilder; one builder connects nodes.
EVCBuilder = ExperimentBuilder


def build_experiment(name, priors=None, algorithms="random", max_trials=float("inf"),
                     pool_size=1, user_args=None, storage=None, working_dir=None, version=None,
                     strategy=None, **branching):
    """Programmatic construction (no CLI): ``build_experiment('exp', {'/lr': 'loguniform(..)'})``."""
    from ..io.resolve_config import get_user
    from .. import __version__
    md = {"user": get_user(), "orion_version": __version__}
    if user_args is not None:
        md["user_args"] = list(user_args)
    if priors is not None:
        md["priors"] = dict(priors)
    config = {"name": name, "metadata": md, "algorithms": algorithms, "max_trials": max_trials,
              "pool_size": pool_size, "working_dir": working_dir}
    if version is not None:
        config["version"] = version
    if strategy is not None:
        config["producer"] = {"strategy": strategy}
    config.update({k: v for k, v in branching.items() if k in BRANCHING_KEYS})
    builder = ExperimentBuilder(storage=storage)
    st = builder.setup_storage(config)

    def merged():
        if not st.fetch_experiments({"name": name}):
            return copy.deepcopy(config)
        try:
            db_cfg = ExperimentView(name, version=version, storage=st).configuration
        except ValueError:
            return copy.deepcopy(config)
        return resolve_config.merge_configs(db_cfg, copy.deepcopy(config))

    try:
        return builder.build_from_config(merged())
    except (DuplicateKeyError, RaceCondition):
        return builder.build_from_config(merged())
