"""Conflicts between a stored experiment configuration and a new one, and their resolutions
(reference: ``src/orion/core/evc/conflicts.py:68-1638``).

``detect_conflicts(old_config, new_config)`` runs every conflict type:

=========================  ====================================  ===============================
conflict                   resolution (marker / flag)            adapter
=========================  ====================================  ===============================
NewDimensionConflict       AddDimensionResolution ``~+``         DimensionAddition
ChangedDimensionConflict   ChangeDimensionResolution ``~+``      DimensionPriorChange
MissingDimensionConflict   RemoveDimensionResolution ``~-``      DimensionDeletion
                           RenameDimensionResolution ``~>new``   DimensionRenaming
AlgorithmConflict          ``--algorithm-change``                AlgorithmChange
CodeConflict               ``--code-change-type {noeffect,...}``  CodeChange (default ``break``)
CommandLineConflict        ``--cli-change-type``                 CommandLineChange
ScriptConfigConflict       ``--config-change-type``              ScriptConfigChange
ExperimentNameConflict     ``--branch NAME`` or version + 1      (none)
=========================  ====================================  ===============================

A resolution's ``repr`` is exactly what a user types to obtain it automatically.
"""
from __future__ import annotations

import copy
import logging
import pprint
import traceback

from ..core.config import config as global_config
from ..io.space_parser import SpaceCmdlineParser
from ..space.builder import SpaceBuilder
from ..space.dims import Dimension
from ..utils.diff import colored_diff
from ..utils.format_trials import standard_param_name
from . import adapters

log = logging.getLogger(__name__)
NO_DEFAULT = Dimension.NO_DEFAULT_VALUE


_STORAGE_OVERRIDE = []


def _storage():
    """The storage of the experiment being configured (``using_storage``), else the
    process-wide one."""
    if _STORAGE_OVERRIDE:
        return _STORAGE_OVERRIDE[-1]
    from ..storage.protocol import get_storage
    return get_storage()


class using_storage:
    """Context: conflict detection/resolution queries go to ``storage``."""

    def __init__(self, storage):
        self.storage = storage

    def __enter__(self):
        _STORAGE_OVERRIDE.append(self.storage)
        return self.storage

    def __exit__(self, *exc):
        _STORAGE_OVERRIDE.pop()


def _create_param(dimension, default_value):
    return dict(name=dimension.name, type=dimension.type, value=default_value)


def _parser(config) -> SpaceCmdlineParser:
    p = SpaceCmdlineParser(global_config.user_script_config)
    state = config.get("metadata", {}).get("parser")
    if state:
        p.set_state_dict(state)
    return p


def _build_extended_user_args(config):
    """User args + ``name~expr`` strings of the user-script config file (for marker search)."""
    user_args = list(config.get("metadata", {}).get("user_args", []) or [])
    parser = _parser(config)
    data = parser.config_file_data if isinstance(parser.config_file_data, dict) else {}
    return user_args + [standard_param_name(k) + str(v) for k, v in data.items()]


def _build_space(config):
    return SpaceBuilder().build(config.get("metadata", {}).get("priors", {}))


def _conflict_types():
    out, stack = [], list(Conflict.__subclasses__())
    while stack:
        cls = stack.pop()
        stack.extend(cls.__subclasses__())
        if not cls.__name__.startswith("_"):
            out.append(cls)
    return sorted(out, key=lambda c: c.__name__)


def detect_conflicts(old_config, new_config) -> "Conflicts":
    conflicts = Conflicts()
    for cls in _conflict_types():
        for c in cls.detect(old_config, new_config):
            conflicts.register(c)
    return conflicts


class Conflicts:
    """A mutable list of conflicts with query/resolve/revert helpers."""

    def __init__(self):
        self.conflicts = []

    def register(self, conflict):
        self.conflicts.append(conflict)

    def revert(self, resolution_or_name):
        name = str(resolution_or_name)
        resolved = self.get_resolved()
        names = [str(c.resolution) for c in resolved]
        resolution = resolved[names.index(name)].resolution
        self.deprecate(resolution.revert())

    def get(self, types=(), dimension_name=None, callback=None):
        def ok(c):
            if callback is not None and not callback(c):
                return False
            if types and not isinstance(c, tuple(types)):
                return False
            if dimension_name is not None and (
                    not hasattr(c, "dimension") or
                    standard_param_name(c.dimension.name) != dimension_name):
                return False
            return True

        found = [c for c in self.conflicts if ok(c)]
        if dimension_name is not None and not found:
            raise ValueError(f"Dimension name '{dimension_name}' not found in conflicts")
        return found

    def get_remaining(self, types=(), dimension_name=None, callback=None):
        return self.get(types, dimension_name,
                        lambda c: not c.is_resolved and (callback is None or callback(c)))

    def get_resolved(self, types=(), dimension_name=None, callback=None):
        return self.get(types, dimension_name,
                        lambda c: c.is_resolved and (callback is None or callback(c)))

    def get_resolutions(self, types=(), dimension_name=None, callback=None):
        seen = []
        for c in self.get_resolved(types, dimension_name, callback):
            if c.resolution is not None and all(c.resolution is not s for s in seen):
                seen.append(c.resolution)
                yield c.resolution

    @property
    def are_resolved(self):
        return all(c.is_resolved for c in self.conflicts)

    def deprecate(self, conflicts):
        for c in conflicts:
            self.conflicts.remove(c)

    def try_resolve(self, conflict, *args, silence_errors=False, **kwargs):
        try:
            resolution = conflict.try_resolve(*args, **kwargs)
        except KeyboardInterrupt:
            raise
        except Exception:  # invalid resolution arguments: the conflict stays open
            conflict.resolution = None
            conflict._is_resolved = None
            if not silence_errors:
                print(traceback.format_exc())
            return None
        if resolution:
            self.conflicts += resolution.new_conflicts
        return resolution


class Conflict:
    @classmethod
    def detect(cls, old_config, new_config):
        return iter(())

    def __init__(self, old_config, new_config):
        self.old_config = old_config
        self.new_config = new_config
        self._is_resolved = False
        self.resolution = None

    @property
    def is_resolved(self):
        return bool(self._is_resolved) or self.resolution is not None

    def get_marked_arguments(self, conflicts):
        return {}

    def try_resolve(self, *args, **kwargs):
        raise NotImplementedError

    @property
    def diff(self):
        return None

    def __repr__(self):  # pragma: no cover - subclasses override
        return type(self).__name__


class Resolution:
    MARKER = None
    ARGUMENT = None

    def __init__(self, conflict):
        self.conflict = conflict
        self.new_conflicts = []
        conflict.resolution = self

    def validate(self, *args, **kwargs):
        try:
            self._validate(*args, **kwargs)
        except Exception:
            self.revert()
            raise

    def _validate(self, *args, **kwargs):
        pass

    @classmethod
    def namespace(cls):
        return cls.ARGUMENT.lstrip("-").replace("-", "_") if cls.ARGUMENT else None

    def revert(self):
        """Un-resolve the conflict; return side-effect conflicts to deprecate."""
        self.conflict.resolution = None
        deprecated = self.new_conflicts
        self.new_conflicts = []
        return deprecated

    def get_adapters(self):
        raise NotImplementedError

    def find_marked_argument(self):
        new_config = self.conflict.new_config
        if self.MARKER:
            for arg in _build_extended_user_args(new_config):
                if arg.lstrip("-").startswith(self.prefix):
                    return arg
            return None
        return new_config.get(self.namespace(), None)

    @property
    def is_marked(self):
        return self.find_marked_argument() not in (None, False)


# ---------------------------------------------------------------------------------------------
class NewDimensionConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        old_space, new_space = _build_space(old_config), _build_space(new_config)
        for name, dim in new_space.items():
            if name not in old_space:
                yield cls(old_config, new_config, dim, dim.get_prior_string())

    def __init__(self, old_config, new_config, dimension, prior):
        super().__init__(old_config, new_config)
        self.dimension, self.prior = dimension, prior

    def try_resolve(self, default_value=NO_DEFAULT):
        if self.is_resolved:
            return None
        return self.AddDimensionResolution(self, default_value)

    @property
    def diff(self):
        return colored_diff("", self.dimension.get_string())

    def __repr__(self):
        return f"New {standard_param_name(self.dimension.name)}"

    class AddDimensionResolution(Resolution):
        MARKER = "~+"

        def __init__(self, conflict, default_value=NO_DEFAULT):
            super().__init__(conflict)
            if default_value is NO_DEFAULT:
                default_value = conflict.dimension.default_value
            else:
                default_value = conflict.dimension.cast(default_value)
            self.validate(default_value)
            self.default_value = default_value

        def _validate(self, default_value):
            if default_value is not NO_DEFAULT and default_value not in self.conflict.dimension:
                raise ValueError(f"Default value `{default_value}` is outside of dimension's prior "
                                 f"interval `{self.conflict.prior}`")

        def get_adapters(self):
            return [adapters.DimensionAddition(_create_param(self.conflict.dimension,
                                                             self.default_value))]

        @property
        def prefix(self):
            return f"{standard_param_name(self.conflict.dimension.name)}{self.MARKER}"

        @property
        def new_prior(self):
            dim = copy.deepcopy(self.conflict.dimension)
            dim._default_value = self.default_value
            return dim.get_prior_string()

        def __repr__(self):
            return f"{self.prefix}{self.new_prior}"


class ChangedDimensionConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        old_space, new_space = _build_space(old_config), _build_space(new_config)
        for name, dim in new_space.items():
            if name not in old_space:
                continue
            new_prior, old_prior = dim.get_prior_string(), old_space[name].get_prior_string()
            if new_prior != old_prior:
                yield cls(old_config, new_config, dim, old_prior, new_prior)

    def __init__(self, old_config, new_config, dimension, old_prior, new_prior):
        super().__init__(old_config, new_config)
        self.dimension, self.old_prior, self.new_prior = dimension, old_prior, new_prior

    def try_resolve(self):
        if self.is_resolved:
            return None
        return self.ChangeDimensionResolution(self)

    @property
    def diff(self):
        return colored_diff(self.old_prior, self.new_prior)

    def __repr__(self):
        n = standard_param_name(self.dimension.name)
        return f"{n}~{self.old_prior} != {n}~{self.new_prior}"

    class ChangeDimensionResolution(Resolution):
        MARKER = "~+"

        def get_adapters(self):
            c = self.conflict
            return [adapters.DimensionPriorChange(c.dimension.name, c.old_prior, c.new_prior)]

        @property
        def prefix(self):
            return f"{standard_param_name(self.conflict.dimension.name)}{self.MARKER}"

        def __repr__(self):
            return f"{self.prefix}{self.conflict.new_prior}"


class MissingDimensionConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        for c in NewDimensionConflict.detect(new_config, old_config):
            yield cls(old_config, new_config, c.dimension, c.prior)

    def __init__(self, old_config, new_config, dimension, prior):
        super().__init__(old_config, new_config)
        self.dimension, self.prior = dimension, prior

    def get_marked_arguments(self, conflicts):
        return self.get_marked_remove_arguments(conflicts) or \
            self.get_marked_rename_arguments(conflicts)

    def get_marked_remove_arguments(self, conflicts):
        if self.is_resolved:
            return {}
        res = copy.deepcopy(self).try_resolve()
        if not res:
            return {}
        arg = res.find_marked_argument()
        if arg:
            val = arg.split(self.RemoveDimensionResolution.MARKER)[1]
            return {"default_value": self.dimension.cast(val) if val else NO_DEFAULT}
        return {}

    def get_marked_rename_arguments(self, conflicts):
        new_dims = conflicts.get([NewDimensionConflict])
        if not new_dims:
            return {}
        res = copy.deepcopy(self).try_resolve(new_dimension_conflict=copy.deepcopy(new_dims[0]))
        if not res:
            return {}
        arg = res.find_marked_argument()
        if arg:
            new_name = "~>".join(arg.split("~>")[1:])
            try:
                target = conflicts.get([NewDimensionConflict], dimension_name=new_name)[0]
            except ValueError as exc:
                if f"Dimension name '{new_name}' not found" not in str(exc):
                    return {}
                raise
            if target.is_resolved:
                conflicts.revert(str(target.resolution))
            return {"new_dimension_conflict": target}
        return {}

    def try_resolve(self, new_dimension_conflict=None, default_value=NO_DEFAULT):
        if self.is_resolved:
            return None
        if new_dimension_conflict:
            return self.RenameDimensionResolution(self, new_dimension_conflict)
        return self.RemoveDimensionResolution(self, default_value)

    @property
    def diff(self):
        return colored_diff(self.dimension.get_string(), "")

    def __repr__(self):
        return f"Missing {standard_param_name(self.dimension.name)}"

    class RenameDimensionResolution(Resolution):
        MARKER = "~>"

        def __init__(self, conflict, new_dimension_conflict):
            super().__init__(conflict)
            self.new_dimension_conflict = new_dimension_conflict
            new_dimension_conflict.resolution = self
            if conflict.prior != new_dimension_conflict.prior:
                self.new_conflicts.append(ChangedDimensionConflict(
                    conflict.old_config, conflict.new_config, new_dimension_conflict.dimension,
                    conflict.prior, new_dimension_conflict.prior))

        def revert(self):
            self.conflict.resolution = None
            self.new_dimension_conflict.resolution = None
            deprecated = self.new_conflicts
            if deprecated:
                deprecated[0]._is_resolved = True
            self.new_conflicts = []
            return deprecated

        def get_adapters(self):
            return [adapters.DimensionRenaming(self.conflict.dimension.name,
                                               self.new_dimension_conflict.dimension.name)]

        @property
        def prefix(self):
            return f"{standard_param_name(self.conflict.dimension.name)}{self.MARKER}"

        def __repr__(self):
            return f"{self.prefix}{standard_param_name(self.new_dimension_conflict.dimension.name)}"

    class RemoveDimensionResolution(Resolution):
        MARKER = "~-"

        def __init__(self, conflict, default_value=NO_DEFAULT):
            super().__init__(conflict)
            if default_value is NO_DEFAULT:
                default_value = conflict.dimension.default_value
            else:
                default_value = conflict.dimension.cast(default_value)
            self.validate(default_value)
            self.default_value = default_value

        def _validate(self, default_value):
            if default_value is not NO_DEFAULT and default_value not in self.conflict.dimension:
                raise ValueError(f"Default value `{default_value}` is outside of dimension's prior "
                                 f"interval `{self.conflict.prior}`")

        def get_adapters(self):
            return [adapters.DimensionDeletion(_create_param(self.conflict.dimension,
                                                             self.default_value))]

        @property
        def prefix(self):
            return f"{standard_param_name(self.conflict.dimension.name)}{self.MARKER}"

        def __repr__(self):
            s = self.prefix
            if self.default_value is not NO_DEFAULT:
                s += repr(self.default_value)
            return s


class AlgorithmConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        if old_config.get("algorithms") != new_config.get("algorithms"):
            yield cls(old_config, new_config)

    def try_resolve(self):
        if self.is_resolved:
            return None
        return self.AlgorithmResolution(self)

    @property
    def diff(self):
        return colored_diff(pprint.pformat(self.old_config.get("algorithms")),
                            pprint.pformat(self.new_config.get("algorithms")))

    def __repr__(self):
        return (f"{pprint.pformat(self.old_config.get('algorithms'))}\n   !=\n"
                f"{pprint.pformat(self.new_config.get('algorithms'))}")

    class AlgorithmResolution(Resolution):
        ARGUMENT = "--algorithm-change"

        def get_adapters(self):
            return [adapters.AlgorithmChange()]

        def __repr__(self):
            return self.ARGUMENT


class _ChangeTypeConflict(Conflict):
    adapter_cls = None
    resolution_cls = None

    def get_marked_arguments(self, conflicts):
        change_type = self.new_config.get(self.resolution_cls.namespace())
        return dict(change_type=change_type or self.adapter_cls.BREAK)

    def try_resolve(self, change_type=None):
        if self.is_resolved:
            return None
        return self.resolution_cls(self, change_type)


class _ChangeTypeResolution(Resolution):
    adapter_cls = None

    def __init__(self, conflict, change_type):
        super().__init__(conflict)
        self.validate(change_type)
        self.type = change_type

    def _validate(self, change_type):
        self.adapter_cls.validate(change_type)

    def get_adapters(self):
        return [self.adapter_cls(self.type)]

    def __repr__(self):
        return f"{self.ARGUMENT} {self.type}"


class CodeConflict(_ChangeTypeConflict):
    adapter_cls = adapters.CodeChange

    @classmethod
    def detect(cls, old_config, new_config):
        old = old_config.get("metadata", {}).get("VCS")
        new = new_config.get("metadata", {}).get("VCS")
        if new and old != new:
            yield cls(old_config, new_config)

    @property
    def diff(self):
        return colored_diff(pprint.pformat(self.old_config["metadata"].get("VCS")),
                            pprint.pformat(self.new_config["metadata"].get("VCS")))

    def __repr__(self):
        old = pprint.pformat(self.old_config["metadata"].get("VCS")).replace("\n", "")
        new = pprint.pformat(self.new_config["metadata"].get("VCS")).replace("\n", "")
        return f"Old hash commit '{old}'  != new hash commit '{new}'"

    class CodeResolution(_ChangeTypeResolution):
        ARGUMENT = "--code-change-type"
        adapter_cls = adapters.CodeChange


CodeConflict.resolution_cls = CodeConflict.CodeResolution


class CommandLineConflict(_ChangeTypeConflict):
    adapter_cls = adapters.CommandLineChange

    @classmethod
    def get_nameless_args(cls, config):
        if not config.get("metadata", {}).get("parser"):
            return ""
        parser = _parser(config)
        priors = parser.priors_to_normal()
        args = {k: a for k, a in parser.parser.arguments.items()
                if k not in priors}
        return " ".join(f"{k} {a}" for k, a in sorted(args.items(), key=lambda x: x[0]))

    @classmethod
    def detect(cls, old_config, new_config):
        if cls.get_nameless_args(old_config) != cls.get_nameless_args(new_config):
            yield cls(old_config, new_config)

    @property
    def diff(self):
        return colored_diff(self.get_nameless_args(self.old_config),
                            self.get_nameless_args(self.new_config))

    def __repr__(self):
        return (f"Old arguments '{self.get_nameless_args(self.old_config)}' != new arguments "
                f"'{self.get_nameless_args(self.new_config)}'")

    class CommandLineResolution(_ChangeTypeResolution):
        ARGUMENT = "--cli-change-type"
        adapter_cls = adapters.CommandLineChange


CommandLineConflict.resolution_cls = CommandLineConflict.CommandLineResolution


class ScriptConfigConflict(_ChangeTypeConflict):
    adapter_cls = adapters.ScriptConfigChange

    @classmethod
    def get_nameless_config(cls, config):
        if not config.get("metadata", {}).get("parser"):
            return {}
        data = _parser(config).config_file_data
        if not isinstance(data, dict):
            return {}
        return {k: v for k, v in data.items()
                if not (isinstance(v, str) and v.startswith("orion~"))}

    @classmethod
    def detect(cls, old_config, new_config):
        if cls.get_nameless_config(old_config) != cls.get_nameless_config(new_config):
            yield cls(old_config, new_config)

    @property
    def diff(self):
        return colored_diff(pprint.pformat(self.get_nameless_config(self.old_config)),
                            pprint.pformat(self.get_nameless_config(self.new_config)))

    def __repr__(self):
        return "Script's configuration file changed"

    class ScriptConfigResolution(_ChangeTypeResolution):
        ARGUMENT = "--config-change-type"
        adapter_cls = adapters.ScriptConfigChange


ScriptConfigConflict.resolution_cls = ScriptConfigConflict.ScriptConfigResolution


class ExperimentNameConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        yield cls(old_config, new_config)

    def get_marked_arguments(self, conflicts):
        new_name = self.new_config.get(self.ExperimentNameResolution.namespace())
        return dict(new_name=new_name) if new_name else {}

    @property
    def username(self):
        return self.new_config["metadata"]["user"]

    def try_resolve(self, new_name=None):
        if self.is_resolved:
            return None
        return self.ExperimentNameResolution(self, new_name)

    def __repr__(self):
        return (f"Experiment name '{self.old_config['name']}' already exist for user "
                f"'{self.username}'")

    class ExperimentNameResolution(Resolution):
        ARGUMENT = "--branch"

        def __init__(self, conflict, new_name):
            super().__init__(conflict)
            self.new_name = new_name
            self.old_name = conflict.old_config["name"]
            self.old_version = conflict.old_config.get("version", 1)
            self.new_version = self.old_version
            self.validate()
            conflict.new_config["name"] = self.new_name
            conflict.new_config["version"] = self.new_version

        def _validate(self):
            if self.new_name is not None and self.new_name != self.old_name:
                if not self._name_is_unique():
                    raise ValueError(f"Cannot branch from {self.old_name} with name "
                                     f"{self.new_name} since it already exists.")
                self.new_version = 1
            elif self._check_for_greater_versions():
                raise ValueError(
                    f"Experiment name '{self.new_name}' already exist for user "
                    f"'{self.conflict.username}' and has children. Version cannot be "
                    "auto-incremented and a new name is required for branching.")
            else:
                self.new_name = self.old_name
                self.new_version = self.conflict.old_config.get("version", 1) + 1

        def _name_is_unique(self):
            q = {"name": self.new_name, "metadata.user": self.conflict.username}
            return len(_storage().fetch_experiments(q)) == 0

        def _check_for_greater_versions(self):
            parent = self.conflict.old_config
            q = {"name": parent["name"], "refers.parent_id": parent["_id"]}
            return bool(_storage().fetch_experiments(q))

        def revert(self):
            self.conflict.new_config["name"] = self.old_name
            self.conflict.new_config["version"] = self.old_version
            return super().revert()

        def get_adapters(self):
            return []

        def __repr__(self):
            return f"{self.ARGUMENT} {self.new_name}"

        @property
        def is_marked(self):
            return True
