"""Resolve the conflicts of a branching event, automatically or one command at a time.

Behaviour contract (reference ``src/orion/core/io/experiment_branch_builder.py:33-310``): every
conflict is first tried with the arguments its markers / flags give; in ``manual_resolution``
mode only the resolutions the user explicitly marked are kept; the remaining methods are the
interactive prompt's commands; ``create_adapters`` chains the adapters of every resolution.

Structure: the auto pass walks the conflicts in registry order (``conflicts.REGISTRY``: names,
then renames before additions); the prompt commands go through two generic entry points --
:meth:`_resolve_single` for the one-per-event conflicts (name, code, command line, script
configuration, algorithm) and :meth:`_resolve_dimension` for the per-dimension ones.
"""
from __future__ import annotations

import logging

from ..space.dims import Dimension
from . import conflicts as C
from .adapters import CompositeAdapter

log = logging.getLogger(__name__)

# prompt command -> the single conflict type it resolves and the keyword of its argument
_SINGLE = {
    "name": (C.ExperimentNameConflict, "new_name"),
    "code": (C.CodeConflict, "change_type"),
    "cli": (C.CommandLineConflict, "change_type"),
    "config": (C.ScriptConfigConflict, "change_type"),
    "algo": (C.AlgorithmConflict, None),
}


class ExperimentBranchBuilder:
    def __init__(self, conflicts: C.Conflicts, branching_configuration=None):
        options = dict(branching_configuration or {})
        if options.pop("auto_resolution", None) is not None:
            log.info("--auto-resolution is deprecated: conflicts are resolved automatically "
                     "unless --manual-resolution is given")
        self.manual_resolution = bool(options.pop("manual_resolution", False))
        self.conflicts = conflicts
        # the branching flags travel with the new configuration (markers read them there)
        self.conflicting_config.update({k: v for k, v in options.items() if v is not None})
        self.resolve_conflicts()

    @property
    def experiment_config(self) -> dict:
        return self.conflicts.conflicts[0].old_config

    @property
    def conflicting_config(self) -> dict:
        return self.conflicts.conflicts[0].new_config

    @property
    def is_resolved(self) -> bool:
        return self.conflicts.are_resolved

    def resolve_conflicts(self, silence_errors=True) -> None:
        """The automatic pass (side conflicts raised on the way are visited too)."""
        pending = sorted(self.conflicts.conflicts, key=lambda c: c.priority)
        seen = set()
        while pending:
            conflict = pending.pop(0)
            if id(conflict) in seen or conflict not in self.conflicts.conflicts:
                continue
            seen.add(id(conflict))
            try:
                args = self.conflicts.marked_arguments(conflict) or {}
            except ValueError as exc:   # a marker naming an unknown dimension
                if not silence_errors:
                    raise
                log.warning("%s: %s", conflict, exc)
                continue
            before = len(self.conflicts.conflicts)
            res = self.conflicts.try_resolve(conflict, silence_errors=silence_errors, **args)
            if res is None:
                continue
            if self.manual_resolution and not res.is_marked:
                self.conflicts.revert(res)
                continue
            pending.extend(self.conflicts.conflicts[before:])

    # -- prompt API ------------------------------------------------------------------------
    def _resolve_single(self, kind, value=None):
        kind_cls, keyword = _SINGLE[kind]
        open_ = self.conflicts.get_remaining([kind_cls])
        if not open_:
            raise RuntimeError(f"No {kind_cls.__name__} to solve")
        kwargs = {keyword: value} if keyword else {}
        return self.conflicts.try_resolve(open_[0], **kwargs)

    def _resolve_dimension(self, types, name, **kwargs):
        return self.conflicts.try_resolve(
            self.conflicts.get_remaining(types, dimension_name=name)[0], **kwargs)

    def change_experiment_name(self, name):
        self._resolve_single("name", name)

    def set_code_change_type(self, change_type):
        self._resolve_single("code", change_type)

    def set_cli_change_type(self, change_type):
        self._resolve_single("cli", change_type)

    def set_script_config_change_type(self, change_type):
        self._resolve_single("config", change_type)

    def set_algo(self):
        self._resolve_single("algo")

    def add_dimension(self, name, default_value=Dimension.NO_DEFAULT_VALUE):
        """Resolve a new (with ``default_value``) or changed dimension ``name``."""
        conflict = self.conflicts.get_remaining(
            [C.NewDimensionConflict, C.ChangedDimensionConflict], dimension_name=name)[0]
        kwargs = ({"default_value": default_value}
                  if isinstance(conflict, C.NewDimensionConflict) else {})
        self.conflicts.try_resolve(conflict, **kwargs)

    def remove_dimension(self, name, default_value=Dimension.NO_DEFAULT_VALUE):
        self._resolve_dimension([C.MissingDimensionConflict], name, default_value=default_value)

    def rename_dimension(self, old_name, new_name):
        old = self.conflicts.get_remaining([C.MissingDimensionConflict], dimension_name=old_name)
        new = self.conflicts.get_remaining([C.NewDimensionConflict], dimension_name=new_name)
        if len(old) != 1 or len(new) != 1:
            raise ValueError(f"ambiguous rename {old_name} -> {new_name}")
        self.conflicts.try_resolve(old[0], new_dimension_conflict=new[0])

    def reset(self, resolution_text):
        self.conflicts.revert(resolution_text)

    def create_adapters(self) -> CompositeAdapter:
        chain = []
        for res in self.conflicts.get_resolutions():
            chain.extend(res.adapters())
        return CompositeAdapter(*chain)
