"""Resolve branching conflicts, automatically or step by step
(reference: ``src/orion/core/io/experiment_branch_builder.py:33-310``).

On construction every conflict is tried with the arguments its markers give
(``get_marked_arguments``); with ``manual_resolution`` only explicitly marked resolutions are kept.
The methods below are the API of the interactive prompt.
"""
from __future__ import annotations

import logging

from ..space.dims import Dimension
from . import conflicts as C
from .adapters import CompositeAdapter

log = logging.getLogger(__name__)


class ExperimentBranchBuilder:
    def __init__(self, conflicts, branching_configuration=None):
        branching_configuration = dict(branching_configuration or {})
        if branching_configuration.pop("auto_resolution", None) is not None:
            log.info("Auto-resolution is deprecated: resolution is automatic unless "
                     "--manual-resolution is given.")
        self.manual_resolution = branching_configuration.pop("manual_resolution", False)
        self.conflicts = conflicts
        self.conflicting_config.update({k: v for k, v in branching_configuration.items()
                                        if v is not None})
        self.resolve_conflicts()

    @property
    def experiment_config(self):
        return self.conflicts.get()[0].old_config

    @property
    def conflicting_config(self):
        return self.conflicts.get()[0].new_config

    def resolve_conflicts(self, silence_errors=True):
        i = 0
        while i < len(self.conflicts.get()):
            conflict = self.conflicts.conflicts[i]
            res = self.conflicts.try_resolve(conflict, silence_errors=silence_errors,
                                             **conflict.get_marked_arguments(self.conflicts))
            if res and self.manual_resolution and not res.is_marked:
                self.conflicts.revert(res)
            i += 1

    @property
    def is_resolved(self):
        return self.conflicts.are_resolved

    def _one(self, types, what):
        remaining = self.conflicts.get_remaining(types)
        if not remaining:
            raise RuntimeError(f"No {what} to solve")
        return remaining[0]

    def change_experiment_name(self, name):
        self.conflicts.try_resolve(self._one([C.ExperimentNameConflict],
                                             "experiment name conflict"), name)

    def set_code_change_type(self, change_type):
        self.conflicts.try_resolve(self._one([C.CodeConflict], "code conflicts"),
                                   change_type=change_type)

    def set_cli_change_type(self, change_type):
        self.conflicts.try_resolve(self._one([C.CommandLineConflict], "command line conflicts"),
                                   change_type)

    def set_script_config_change_type(self, change_type):
        self.conflicts.try_resolve(self._one([C.ScriptConfigConflict],
                                             "script's config conflicts"), change_type)

    def set_algo(self):
        self.conflicts.try_resolve(self._one([C.AlgorithmConflict], "algo conflict"))

    def add_dimension(self, name, default_value=Dimension.NO_DEFAULT_VALUE):
        conflict = self.conflicts.get_remaining(
            [C.NewDimensionConflict, C.ChangedDimensionConflict], dimension_name=name)[0]
        if isinstance(conflict, C.NewDimensionConflict):
            self.conflicts.try_resolve(conflict, default_value=default_value)
        else:
            self.conflicts.try_resolve(conflict)

    def remove_dimension(self, name, default_value=Dimension.NO_DEFAULT_VALUE):
        conflict = self.conflicts.get_remaining([C.MissingDimensionConflict],
                                                dimension_name=name)[0]
        self.conflicts.try_resolve(conflict, default_value=default_value)

    def rename_dimension(self, old_name, new_name):
        old = self.conflicts.get_remaining([C.MissingDimensionConflict], dimension_name=old_name)
        new = self.conflicts.get_remaining([C.NewDimensionConflict], dimension_name=new_name)
        if len(old) != 1 or len(new) != 1:
            raise ValueError("ambiguous rename")
        self.conflicts.try_resolve(old[0], new_dimension_conflict=new[0])

    def reset(self, name):
        self.conflicts.revert(name)

    def create_adapters(self) -> CompositeAdapter:
        adapters = []
        for res in self.conflicts.get_resolutions():
            adapters += res.get_adapters()
        return CompositeAdapter(*adapters)
