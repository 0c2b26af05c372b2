"""Experiments: a named, versioned search over one space with one algorithm
(reference: ``src/orion/core/worker/experiment.py:37-744``).

Document::

    {_id, name, version, metadata: {user, datetime, orion_version, user_script, user_args,
     VCS, parser, priors}, refers: {root_id, parent_id, adapter}, pool_size, max_trials,
     working_dir, algorithms: {name: {params}}, producer: {strategy: ...}}

``Experiment(name, version=None)`` loads the latest (or requested) version from storage;
``configure(config)`` validates a configuration, detects conflicts with the stored version,
branches through the experiment version control (EVC) when needed -- automatically from markers
and branching flags, or through the interactive prompt on a TTY -- and persists the result.
A race on the unique ``(name, version)`` index surfaces as ``RaceCondition``/``DuplicateKeyError``
and is retried once by the builder.

Trials: ``register_trial`` (dedup by md5 ``_id``), ``reserve_trial`` (lost-trial sweep, then the
atomic reserve), ``update_completed_trial``, ``register_lie``; ``is_done`` (completed >=
max_trials or the algorithm is done), ``is_broken`` (broken >= worker.max_broken), ``stats``.
"""
from __future__ import annotations

import copy
import datetime
import logging
import sys
from typing import List, Optional

from ..algo.primary import PrimaryAlgo
from ..space.builder import SpaceBuilder
from ..storage.database import DuplicateKeyError
from ..storage.protocol import ReadOnlyStorage, get_storage
from ..utils.exceptions import RaceCondition
from ..worker.strategy import BaseParallelStrategy, create_strategy
from .config import config as global_config
from .trial import Trial

log = logging.getLogger(__name__)


def _get_user():
    from ..io.resolve_config import get_user
    return get_user()


class Experiment:
    __slots__ = ("name", "refers", "metadata", "pool_size", "max_trials", "version", "algorithms",
                 "producer", "working_dir", "_init_done", "_id", "_node", "_storage")
    non_branching_attrs = ("pool_size", "max_trials")

    def __init__(self, name, user=None, version=None, storage=None):
        self._init_done = False
        self._id = None
        self.name = name
        self._node = None
        self.refers = {}
        self.metadata = {"user": user or _get_user()}
        self.pool_size = None
        self.max_trials = None
        self.algorithms = None
        self.working_dir = None
        self.producer = {"strategy": None}
        self.version = 1
        self._storage = storage if storage is not None else get_storage()

        configs = self._storage.fetch_experiments({"name": name})
        if configs:
            max_version = max(c.get("version", 1) for c in configs)
            if version is None:
                self.version = max_version
            else:
                if version > max_version:
                    log.warning("Version %s was specified but most recent version is only %s. "
                                "Using %s.", version, max_version, max_version)
                self.version = min(version, max_version)
            configs = [c for c in configs if c.get("version", 1) == self.version]
            cfg = sorted(configs, key=lambda c: c["metadata"].get("datetime") or
                         datetime.datetime.min, reverse=True)[0]
            populate_priors(cfg["metadata"])
            for attr in self.__slots__:
                if not attr.startswith("_") and attr in cfg:
                    setattr(self, attr, cfg[attr])
            self._id = cfg["_id"]

    # -- trials -------------------------------------------------------------------------------
    def fetch_trials(self, with_evc_tree=False) -> List[Trial]:
        return self._select_evc_call(with_evc_tree, "fetch_trials")

    def fetch_trials_by_status(self, status, with_evc_tree=False):
        return self._select_evc_call(with_evc_tree, "fetch_trials_by_status", status)

    def fetch_noncompleted_trials(self, with_evc_tree=False):
        return self._select_evc_call(with_evc_tree, "fetch_noncompleted_trials")

    def fetch_pending_trials(self):
        return self._storage.fetch_pending_trials(self)

    def _select_evc_call(self, with_evc_tree, function, *args):
        if self._node is not None and with_evc_tree:
            return getattr(self._node, function)(*args)
        return getattr(self._storage, function)(self, *args)

    def get_trial(self, trial=None, uid=None):
        return self._storage.get_trial(trial, uid)

    def connect_to_version_control_tree(self, node):
        self._node = node

    def retrieve_result(self, trial, *args, **kwargs):
        return self._storage.retrieve_result(trial, *args, **kwargs)

    def set_trial_status(self, *args, **kwargs):
        return self._storage.set_trial_status(*args, **kwargs)

    def reserve_trial(self, score_handle=None) -> Optional[Trial]:
        if score_handle is not None:
            log.warning("Argument `score_handle` is deprecated")
        self.fix_lost_trials()
        return self._storage.reserve_trial(self)

    def fix_lost_trials(self):
        """Reserved trials whose heartbeat went stale become 'interrupted' (re-reservable)."""
        from ..storage.protocol import FailedUpdate
        for trial in self._storage.fetch_lost_trials(self):
            try:
                self._storage.set_trial_status(trial, status="interrupted")
            except FailedUpdate:
                log.debug("lost trial %s was recovered by another worker", trial.id)

    def update_completed_trial(self, trial: Trial, results_file=None):
        trial.status = "completed"
        trial.end_time = datetime.datetime.utcnow()
        if results_file is not None:
            self._storage.retrieve_result(trial, results_file)
        self._storage.push_trial_results(trial)

    def register_lie(self, lying_trial: Trial):
        lying_trial.status = "completed"
        lying_trial.end_time = datetime.datetime.utcnow()
        self._storage.register_lie(lying_trial)

    def register_trial(self, trial: Trial):
        trial.experiment = self._id
        trial.status = "new"
        trial.submit_time = datetime.datetime.utcnow()
        self._storage.register_trial(trial)

    def register_trials(self, trials: List[Trial]) -> List[Trial]:
        """Register many trials; duplicates of already registered ones are skipped."""
        stamp = datetime.datetime.utcnow()
        done = []
        for t in trials:
            t.experiment = self._id
            t.status = "new"
            t.submit_time = stamp
            try:
                self._storage.register_trial(t)
                done.append(t)
            except DuplicateKeyError:
                log.debug("duplicate trial %s skipped", t.id)
        return done

    # -- properties ---------------------------------------------------------------------------
    @property
    def id(self):
        return self._id

    @property
    def node(self):
        return self._node

    @property
    def storage(self):
        return self._storage

    @property
    def is_done(self) -> bool:
        n = self._storage.count_completed_trials(self)
        return bool(n >= self.max_trials or (self._init_done and self.algorithms.is_done))

    @property
    def is_broken(self) -> bool:
        return self._storage.count_broken_trials(self) >= global_config.worker.max_broken

    @property
    def space(self):
        return self.algorithms.space if self._init_done else None

    @property
    def configuration(self) -> dict:
        cfg = {}
        for attr in self.__slots__:
            if attr.startswith("_"):
                continue
            value = getattr(self, attr)
            if self._init_done and attr == "algorithms":
                value = value.configuration
            elif attr == "refers":
                value = copy.copy(value)
                adapter = value.get("adapter")
                if adapter is not None and not isinstance(adapter, list):
                    value["adapter"] = adapter.configuration
            elif attr == "producer":
                value = copy.copy(value)
                strat = value.get("strategy")
                if isinstance(strat, BaseParallelStrategy):
                    value["strategy"] = strat.configuration
            cfg[attr] = value
        return copy.deepcopy(cfg)

    @property
    def stats(self) -> dict:
        completed = self.fetch_trials_by_status("completed")
        if not completed:
            return {}
        best = min(completed, key=lambda t: t.objective.value)
        start = self.metadata.get("datetime")
        finish = max([t.end_time for t in completed if t.end_time] or [start])
        stats = {"trials_completed": len(completed), "best_trials_id": best.id,
                 "best_evaluation": best.objective.value, "start_time": start,
                 "finish_time": finish}
        stats["duration"] = (finish - start) if (finish and start) else None
        return stats

    # -- configuration ------------------------------------------------------------------------
    def configure(self, config, enable_branching=True, enable_update=True):
        """Validate ``config``, branch if it conflicts with the stored version, persist."""
        from ..evc.conflicts import using_storage
        with using_storage(self._storage):
            return self._configure(config, enable_branching, enable_update)

    def _configure(self, config, enable_branching=True, enable_update=True):
        from ..evc.conflicts import ExperimentNameConflict, detect_conflicts
        log.debug("configuring (name: %s)", config["name"])
        if self._init_done:
            raise RuntimeError("Configuration is done; cannot reset an Experiment.")
        if self._id is not None and "datetime" not in config.get("metadata", {}):
            raise DuplicateKeyError("Cannot register an existing experiment with a new config")

        experiment = Experiment(self.name, version=self.version, storage=self._storage)
        experiment._instantiate_config(self.configuration)
        experiment._instantiate_config(config)
        experiment._init_done = True

        branching = dict(config.get("branching") or {})
        if self._id is None:
            if config["name"] != self.name or \
                    config["metadata"]["user"] != self.metadata["user"]:
                raise ValueError("Configuration given is inconsistent with this Experiment.")
            must_branch = True
        else:
            current = self.configuration
            current["_id"] = self._id
            conflicts = detect_conflicts(current, experiment.configuration)
            must_branch = len(conflicts.get()) > 1 or bool(branching.get("branch"))
            name_conflict = conflicts.get([ExperimentNameConflict])[0]
            if not name_conflict.is_resolved and not config.get("version"):
                raise RaceCondition("There was likely a race condition during version increment.")
            if must_branch and not enable_branching:
                raise ValueError("Configuration is different and generate a branching event")
            if must_branch:
                experiment._branch_config(conflicts, branching)

        final = experiment.configuration
        self._instantiate_config(final)
        self._init_done = True
        if not enable_update:
            return
        if must_branch:
            final["metadata"]["datetime"] = datetime.datetime.utcnow()
            self.metadata["datetime"] = final["metadata"]["datetime"]
            final.pop("_id", None)
            try:
                self._storage.create_experiment(final)
            except DuplicateKeyError:
                self._init_done = False    # lost the race: this object was never registered
                raise
            self._id = final["_id"]
            if self.refers.get("parent_id") is None:
                self.refers["root_id"] = self._id
                self._storage.update_experiment(self, refers=self.configuration["refers"])
        else:
            final.pop("name")
            self._storage.update_experiment(self, **final)

    def _instantiate_config(self, config):
        from ..evc.adapters import Adapter, BaseAdapter
        for section, value in config.items():
            if section not in self.__slots__ or section.startswith("_"):
                continue
            setattr(self, section, copy.deepcopy(value) if isinstance(value, dict) else value)
        try:
            priors = config["metadata"]["priors"]
        except (KeyError, TypeError):
            priors = None
        if priors is not None:
            space = SpaceBuilder().build(priors)
            if not space:
                raise ValueError("Parameter space is empty. There is nothing to optimize.")
            algo_cfg = self.algorithms
            if isinstance(algo_cfg, PrimaryAlgo):
                algo_cfg = algo_cfg.configuration
            self.algorithms = PrimaryAlgo(space, algo_cfg or "random")
        self.refers.setdefault("parent_id", None)
        self.refers.setdefault("root_id", self._id)
        self.refers.setdefault("adapter", [])
        if not isinstance(self.refers.get("adapter"), BaseAdapter):
            self.refers["adapter"] = Adapter.build(self.refers["adapter"])
        if not isinstance(self.producer, dict):
            self.producer = {"strategy": self.producer}
        strat = self.producer.get("strategy")
        if not strat:
            self.producer = {"strategy": create_strategy("MaxParallelStrategy")}
        elif not isinstance(strat, BaseParallelStrategy):
            self.producer = {"strategy": create_strategy(strat)}

    def _branch_config(self, conflicts, branching):
        from ..evc.branch_builder import ExperimentBranchBuilder
        from ..evc.prompt import BranchingPrompt
        brancher = ExperimentBranchBuilder(conflicts, branching)
        if not brancher.is_resolved or brancher.manual_resolution:
            prompt = BranchingPrompt(brancher)
            if not sys.__stdin__ or not sys.__stdin__.isatty():
                raise ValueError("Configuration is different and generates a branching event:\n"
                                 f"{prompt.get_status()}")
            prompt.cmdloop()
            if prompt.abort or not brancher.is_resolved:
                sys.exit()
        adapter = brancher.create_adapters()
        self._instantiate_config(brancher.conflicting_config)
        self.refers["adapter"] = adapter
        self.refers["parent_id"] = self._id

    def __repr__(self):
        return (f"Experiment(name={self.name}, metadata.user={self.metadata.get('user')}, "
                f"version={self.version})")


def populate_priors(metadata: dict) -> None:
    """Backward compatibility: derive ``parser``/``priors`` from ``user_args`` for documents
    written by versions that did not store them (reference ``core/utils/backward.py:17-27``)."""
    if "user_args" not in metadata:
        return
    if "parser" in metadata and "priors" in metadata:
        return
    from ..io.space_parser import SpaceCmdlineParser
    parser = SpaceCmdlineParser(global_config.user_script_config)
    parser.parse(metadata["user_args"])
    metadata["parser"] = parser.get_state_dict()
    metadata["priors"] = dict(parser.priors)


class ExperimentView:
    """Read-only experiment (reference ``experiment.py:673-744``)."""

    __slots__ = ("_experiment",)
    valid_attributes = (["_id", "name", "refers", "metadata", "pool_size", "max_trials",
                         "version", "working_dir", "producer"] +
                        ["id", "node", "is_done", "space", "algorithms", "stats", "configuration",
                         "is_broken"] +
                        ["fetch_trials", "fetch_trials_by_status", "fetch_noncompleted_trials",
                         "connect_to_version_control_tree", "get_trial", "storage"])

    def __init__(self, name, user=None, version=None, storage=None):
        from ..evc.adapters import Adapter, BaseAdapter
        exp = Experiment(name, user, version, storage=storage)
        if exp.id is None:
            raise ValueError(f"No experiment with given name '{exp.name}' for user "
                             f"'{exp.metadata['user']}' inside database, no view can be created.")
        object.__setattr__(self, "_experiment", exp)
        try:
            exp._instantiate_config(exp.configuration)
            exp._init_done = True
        except Exception as exc:  # the view stays usable for trial/stat queries
            log.debug("view of %s could not build its space/algorithm: %s", name, exc)
            exp.refers.setdefault("parent_id", None)
            exp.refers.setdefault("root_id", exp._id)
            exp.refers.setdefault("adapter", [])
            if not isinstance(exp.refers.get("adapter"), BaseAdapter):
                exp.refers["adapter"] = Adapter.build(exp.refers["adapter"])
        exp._storage = ReadOnlyStorage(exp._storage)

    def __getattr__(self, name):
        if name not in self.valid_attributes:
            raise AttributeError(f"Cannot access attribute {name} on view-only experiments.")
        return getattr(self._experiment, name)

    def __repr__(self):
        exp = self._experiment
        return (f"ExperimentView(name={exp.name}, metadata.user={exp.metadata.get('user')}, "
                f"version={exp.version})")
