"""Conflicts between a stored experiment configuration and a new one, and their resolutions.

Behaviour contract: the reference's ``src/orion/core/evc/conflicts.py:68-1638`` -- which
differences are conflicts, which resolutions solve them, the markers / flags a user types to
choose a resolution, the resulting adapters, and each resolution's textual form (its ``repr``
is what a user types to get it).  The structure is this package's own:

* conflict types register themselves in :data:`REGISTRY` with a *priority*; ``detect_conflicts``
  runs the detectors in that order (renames are claimed before additions are auto-resolved);
* the markers of a configuration (``name~+prior``, ``name~-[default]``, ``name~>new``) are
  parsed **once** into a :class:`Markers` index that every conflict consults, instead of each
  resolution re-scanning the user arguments;
* resolutions are top-level classes carrying their marker / flag, their adapter recipe and
  their side conflicts; :data:`FLAGS` gives the CLI flags (``cli/evc.py``).

=========================  ================================  ==============================
conflict                   resolution (marker / flag)        adapter
=========================  ================================  ==============================
ExperimentNameConflict     ``--branch NAME`` or version + 1  (none)
MissingDimensionConflict   ``~-`` remove / ``~>new`` rename  DimensionDeletion / Renaming
NewDimensionConflict       ``~+`` add                        DimensionAddition
ChangedDimensionConflict   ``~+`` change                     DimensionPriorChange
AlgorithmConflict          ``--algorithm-change``            AlgorithmChange
CodeConflict               ``--code-change-type``            CodeChange (default ``break``)
CommandLineConflict        ``--cli-change-type``             CommandLineChange
ScriptConfigConflict       ``--config-change-type``          ScriptConfigChange
=========================  ================================  ==============================
"""
from __future__ import annotations

import copy
import logging
import pprint
import re
import traceback
from typing import Dict, List, Optional

from ..core.config import config as global_config
from ..io.space_parser import SpaceCmdlineParser
from ..space.builder import SpaceBuilder
from ..space.dims import Dimension
from ..utils.diff import colored_diff
from ..utils.format_trials import standard_param_name
from . import adapters as A

log = logging.getLogger(__name__)
NO_DEFAULT = Dimension.NO_DEFAULT_VALUE


# ---------------------------------------------------------------------------------- storage
_STORAGES: list = []


def _storage():
    """Storage of the experiment being configured (:class:`using_storage`), else the global."""
    if _STORAGES:
        return _STORAGES[-1]
    from ..storage.protocol import get_storage
    return get_storage()


class using_storage:
    """Context: name-conflict queries (uniqueness, children) go to ``storage``."""

    def __init__(self, storage):
        self.storage = storage

    def __enter__(self):
        _STORAGES.append(self.storage)
        return self.storage

    def __exit__(self, *exc):
        _STORAGES.pop()


# ---------------------------------------------------------------------------------- markers
class Markers:
    """The EVC markers of a configuration, by standard dimension name (no leading ``/``):
    ``{"y": ("-", "")}`` for ``--y~-``, ``("-", "0.5")`` for ``--y~-0.5``, ``(">", "z")`` for
    ``--y~>z``, ``("+", "uniform(0, 1)")`` for ``--y~+uniform(0, 1)``.  Sources: the user
    arguments and the user-script configuration file (``name: orion~+prior`` values)."""

    _ARG = re.compile(r"^-*([^~=\s]+)~([+\->])(.*)$", re.S)

    def __init__(self, config: dict):
        self.config = config
        self.marks: Dict[str, tuple] = {}
        meta = config.get("metadata", {}) or {}
        for arg in meta.get("user_args", []) or []:
            self._add(str(arg))
        for name, value in _file_values(config).items():
            if isinstance(value, str) and "~" in value:
                self._add(name + value[value.index("~"):])

    def _add(self, text):
        m = self._ARG.match(text)
        if m:
            self.marks.setdefault(standard_param_name(m.group(1)), (m.group(2), m.group(3)))

    def get(self, dimension_name: str, marker: str) -> Optional[str]:
        """The text after ``marker`` for dimension ``dimension_name``, or None."""
        hit = self.marks.get(standard_param_name(dimension_name))
        return hit[1] if hit is not None and hit[0] == marker else None

    def flag(self, namespace: str):
        return self.config.get(namespace)


def _user_parser(config) -> SpaceCmdlineParser:
    p = SpaceCmdlineParser(global_config.user_script_config)
    state = (config.get("metadata", {}) or {}).get("parser")
    if state:
        p.set_state_dict(state)
    return p


def _file_values(config) -> dict:
    """Flattened ``{"/a/b": value}`` of the user-script configuration file."""
    data = _user_parser(config).config_file_data
    out = {}

    def walk(node, path):
        if isinstance(node, dict):
            for k, v in node.items():
                walk(v, f"{path}/{k}")
        else:
            out[path] = node
    if isinstance(data, dict):
        walk(data, "")
    return out


def _space(config):
    return SpaceBuilder().build((config.get("metadata", {}) or {}).get("priors", {}))


# ---------------------------------------------------------------------------------- registry
REGISTRY: List[type] = []


def _register(priority: int):
    def deco(cls):
        cls.priority = priority
        REGISTRY.append(cls)
        REGISTRY.sort(key=lambda c: c.priority)
        return cls
    return deco


def detect_conflicts(old_config, new_config) -> "Conflicts":
    """Every conflict between the stored ``old_config`` and ``new_config`` (the name conflict
    always: the new configuration needs a new version or a new name)."""
    found = Conflicts(markers=Markers(new_config))
    for cls in REGISTRY:
        for c in cls.detect(old_config, new_config):
            found.register(c)
    return found


class Conflicts:
    """The conflicts of one branching event, with queries, resolution and revert."""

    def __init__(self, markers: Optional[Markers] = None):
        self.conflicts: list = []
        self.markers = markers

    def register(self, conflict):
        self.conflicts.append(conflict)

    def deprecate(self, conflicts):
        for c in conflicts:
            self.conflicts.remove(c)

    def get(self, types=(), dimension_name=None, callback=None):
        types = tuple(types)
        out = [c for c in self.conflicts
               if (not types or isinstance(c, types))
               and (callback is None or callback(c))
               and (dimension_name is None or
                    (hasattr(c, "dimension") and
                     standard_param_name(c.dimension.name) == dimension_name))]
        if dimension_name is not None and not out:
            raise ValueError(f"Dimension name '{dimension_name}' not found in conflicts")
        return out

    def get_remaining(self, types=(), dimension_name=None, callback=None):
        return self.get(types, dimension_name,
                        lambda c: not c.is_resolved and (callback is None or callback(c)))

    def get_resolved(self, types=(), dimension_name=None, callback=None):
        return self.get(types, dimension_name,
                        lambda c: c.is_resolved and (callback is None or callback(c)))

    def get_resolutions(self, types=(), dimension_name=None, callback=None):
        """Distinct resolutions of the resolved conflicts (a rename resolves two)."""
        seen = set()
        for c in self.get_resolved(types, dimension_name, callback):
            r = c.resolution
            if r is not None and id(r) not in seen:
                seen.add(id(r))
                yield r

    @property
    def are_resolved(self) -> bool:
        return all(c.is_resolved for c in self.conflicts)

    def try_resolve(self, conflict, *args, silence_errors=False, **kwargs):
        """Resolve ``conflict``; invalid arguments leave it open (traceback printed unless
        ``silence_errors``).  Side conflicts a resolution raises join the list."""
        try:
            resolution = conflict.try_resolve(*args, **kwargs)
        except KeyboardInterrupt:
            raise
        except Exception:
            conflict.resolution = None
            if not silence_errors:
                print(traceback.format_exc())
            return None
        if resolution is not None:
            self.conflicts.extend(resolution.side_conflicts)
        return resolution

    def revert(self, resolution_or_text):
        """Undo a resolution (the object or its text, as ``status`` prints it)."""
        text = str(resolution_or_text)
        for r in self.get_resolutions():
            if r is resolution_or_text or str(r) == text:
                self.deprecate(r.revert())
                return
        raise ValueError(f"no resolution '{text}' to revert")

    def marked_arguments(self, conflict) -> Optional[dict]:
        """The arguments the user's markers / flags give ``conflict`` (None: nothing marked,
        resolve with defaults)."""
        markers = self.markers or Markers(conflict.new_config)
        return conflict.marked_arguments(markers, self)


# ---------------------------------------------------------------------------------- base types
class Conflict:
    priority = 100

    def __init__(self, old_config, new_config):
        self.old_config = old_config
        self.new_config = new_config
        self.resolution = None

    @classmethod
    def detect(cls, old_config, new_config):
        return ()

    @property
    def is_resolved(self) -> bool:
        return self.resolution is not None

    def marked_arguments(self, markers: Markers, conflicts: Conflicts) -> Optional[dict]:
        return None

    def try_resolve(self, *args, **kwargs):
        """The resolution, or None when already resolved; raises on invalid arguments."""
        if self.is_resolved:
            return None
        return self._resolve(*args, **kwargs)

    def _resolve(self, *args, **kwargs):
        raise NotImplementedError

    @property
    def diff(self):
        return None


class Resolution:
    marker: Optional[str] = None     # dimension marker character ('+', '-', '>')
    flag: Optional[str] = None       # CLI flag

    def __init__(self, conflict):
        self.conflict = conflict
        self.side_conflicts: list = []
        conflict.resolution = self

    @classmethod
    def namespace(cls) -> Optional[str]:
        return cls.flag.lstrip("-").replace("-", "_") if cls.flag else None

    def _fail(self, message):
        self.revert()
        raise ValueError(message)

    def revert(self) -> list:
        """Re-open the conflict(s); returns the side conflicts to deprecate."""
        self.conflict.resolution = None
        side, self.side_conflicts = self.side_conflicts, []
        return side

    def adapters(self) -> list:
        return []

    def get_adapters(self) -> list:
        return self.adapters()

    @property
    def is_marked(self) -> bool:
        """Whether the user explicitly asked for this resolution (kept in manual mode)."""
        markers = Markers(self.conflict.new_config)
        if self.marker is not None:
            return markers.get(self.conflict.dimension.name, self.marker) is not None
        return bool(markers.flag(self.namespace()))


def _dim_label(dimension) -> str:
    return standard_param_name(dimension.name)


def _checked_default(dimension, value, prior):
    """``value`` cast to ``dimension`` (its own default when NO_DEFAULT), validated."""
    value = dimension.default_value if value is NO_DEFAULT else dimension.cast(value)
    if value is not NO_DEFAULT and value not in dimension:
        raise ValueError(f"Default value `{value}` is outside of dimension's prior interval "
                         f"`{prior}`")
    return value


def _as_param(dimension, value) -> dict:
    return {"name": dimension.name, "type": dimension.type, "value": value}


# ---------------------------------------------------------------------------------- dimensions
class AddDimensionResolution(Resolution):
    marker = "+"

    def __init__(self, conflict, default_value=NO_DEFAULT):
        super().__init__(conflict)
        try:
            self.default_value = _checked_default(conflict.dimension, default_value,
                                                  conflict.prior)
        except ValueError as exc:
            self._fail(str(exc))

    def adapters(self):
        return [A.DimensionAddition(_as_param(self.conflict.dimension, self.default_value))]

    @property
    def new_prior(self) -> str:
        dim = copy.deepcopy(self.conflict.dimension)
        dim._default_value = self.default_value
        return dim.get_prior_string()

    def __repr__(self):
        return f"{_dim_label(self.conflict.dimension)}~+{self.new_prior}"


class ChangeDimensionResolution(Resolution):
    marker = "+"

    def adapters(self):
        c = self.conflict
        return [A.DimensionPriorChange(c.dimension.name, c.old_prior, c.new_prior)]

    def __repr__(self):
        return f"{_dim_label(self.conflict.dimension)}~+{self.conflict.new_prior}"


class RemoveDimensionResolution(Resolution):
    marker = "-"

    def __init__(self, conflict, default_value=NO_DEFAULT):
        super().__init__(conflict)
        try:
            self.default_value = _checked_default(conflict.dimension, default_value,
                                                  conflict.prior)
        except ValueError as exc:
            self._fail(str(exc))

    def adapters(self):
        return [A.DimensionDeletion(_as_param(self.conflict.dimension, self.default_value))]

    def __repr__(self):
        text = f"{_dim_label(self.conflict.dimension)}~-"
        return text if self.default_value is NO_DEFAULT else text + repr(self.default_value)


class RenameDimensionResolution(Resolution):
    """Resolves a missing dimension and a new one together; a prior difference between them
    becomes a side :class:`ChangedDimensionConflict`."""
    marker = ">"

    def __init__(self, conflict, new_dimension_conflict):
        if new_dimension_conflict.is_resolved:
            raise ValueError(f"dimension '{_dim_label(new_dimension_conflict.dimension)}' is "
                             "already resolved; reset it before renaming onto it")
        super().__init__(conflict)
        self.target = new_dimension_conflict
        new_dimension_conflict.resolution = self
        if conflict.prior != new_dimension_conflict.prior:
            self.side_conflicts.append(ChangedDimensionConflict(
                conflict.old_config, conflict.new_config, new_dimension_conflict.dimension,
                conflict.prior, new_dimension_conflict.prior))

    @property
    def new_dimension_conflict(self):
        return self.target

    def revert(self):
        self.target.resolution = None
        return super().revert()

    def adapters(self):
        return [A.DimensionRenaming(self.conflict.dimension.name, self.target.dimension.name)]

    def __repr__(self):
        return f"{_dim_label(self.conflict.dimension)}~>{_dim_label(self.target.dimension)}"


def _new_dims(old_config, new_config):
    old, new = _space(old_config), _space(new_config)
    return [(name, dim) for name, dim in new.items() if name not in old]


@_register(10)
class MissingDimensionConflict(Conflict):
    """A dimension of the stored configuration is absent from the new one."""

    def __init__(self, old_config, new_config, dimension, prior):
        super().__init__(old_config, new_config)
        self.dimension, self.prior = dimension, prior

    @classmethod
    def detect(cls, old_config, new_config):
        for _, dim in _new_dims(new_config, old_config):
            yield cls(old_config, new_config, dim, dim.get_prior_string())

    def marked_arguments(self, markers, conflicts):
        removal = markers.get(self.dimension.name, "-")
        if removal is not None:
            return {"default_value": self.dimension.cast(removal) if removal else NO_DEFAULT}
        target = markers.get(self.dimension.name, ">")
        if target is None:
            return None
        found = conflicts.get([NewDimensionConflict], dimension_name=standard_param_name(target))
        if found[0].is_resolved:        # claimed by an automatic addition: the rename wins
            conflicts.revert(found[0].resolution)
        return {"new_dimension_conflict": found[0]}

    def _resolve(self, new_dimension_conflict=None, default_value=NO_DEFAULT):
        if new_dimension_conflict is not None:
            return RenameDimensionResolution(self, new_dimension_conflict)
        return RemoveDimensionResolution(self, default_value)

    @property
    def diff(self):
        return colored_diff(self.dimension.get_string(), "")

    def __repr__(self):
        return f"Missing {_dim_label(self.dimension)}"


@_register(20)
class NewDimensionConflict(Conflict):
    """The new configuration has a dimension the stored one does not."""

    def __init__(self, old_config, new_config, dimension, prior):
        super().__init__(old_config, new_config)
        self.dimension, self.prior = dimension, prior

    @classmethod
    def detect(cls, old_config, new_config):
        for _, dim in _new_dims(old_config, new_config):
            yield cls(old_config, new_config, dim, dim.get_prior_string())

    def _resolve(self, default_value=NO_DEFAULT):
        return AddDimensionResolution(self, default_value)

    @property
    def diff(self):
        return colored_diff("", self.dimension.get_string())

    def __repr__(self):
        return f"New {_dim_label(self.dimension)}"


@_register(30)
class ChangedDimensionConflict(Conflict):
    """A dimension's prior differs between the two configurations."""

    def __init__(self, old_config, new_config, dimension, old_prior, new_prior):
        super().__init__(old_config, new_config)
        self.dimension, self.old_prior, self.new_prior = dimension, old_prior, new_prior

    @classmethod
    def detect(cls, old_config, new_config):
        old = _space(old_config)
        for name, dim in _space(new_config).items():
            if name in old:
                before, after = old[name].get_prior_string(), dim.get_prior_string()
                if before != after:
                    yield cls(old_config, new_config, dim, before, after)

    def _resolve(self):
        return ChangeDimensionResolution(self)

    @property
    def diff(self):
        return colored_diff(self.old_prior, self.new_prior)

    def __repr__(self):
        n = _dim_label(self.dimension)
        return f"{n}~{self.old_prior} != {n}~{self.new_prior}"


# ---------------------------------------------------------------------------------- algorithm
class AlgorithmResolution(Resolution):
    flag = "--algorithm-change"

    def adapters(self):
        return [A.AlgorithmChange()]

    def __repr__(self):
        return self.flag


@_register(40)
class AlgorithmConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        if old_config.get("algorithms") != new_config.get("algorithms"):
            yield cls(old_config, new_config)

    def _resolve(self):
        return AlgorithmResolution(self)

    def _pair(self):
        return (pprint.pformat(self.old_config.get("algorithms")),
                pprint.pformat(self.new_config.get("algorithms")))

    @property
    def diff(self):
        return colored_diff(*self._pair())

    def __repr__(self):
        old, new = self._pair()
        return f"{old}\n   !=\n{new}"


# ---------------------------------------------------------------------------------- typed changes
class _TypedChangeResolution(Resolution):
    adapter_cls = None

    def __init__(self, conflict, change_type):
        super().__init__(conflict)
        try:
            self.adapter_cls.validate(change_type)
        except ValueError as exc:
            self._fail(str(exc))
        self.type = change_type

    def adapters(self):
        return [self.adapter_cls(self.type)]

    def __repr__(self):
        return f"{self.flag} {self.type}"


class CodeResolution(_TypedChangeResolution):
    flag = "--code-change-type"
    adapter_cls = A.CodeChange


class CommandLineResolution(_TypedChangeResolution):
    flag = "--cli-change-type"
    adapter_cls = A.CommandLineChange


class ScriptConfigResolution(_TypedChangeResolution):
    flag = "--config-change-type"
    adapter_cls = A.ScriptConfigChange


class _TypedChangeConflict(Conflict):
    """A change outside the search space: resolved with a change type (default ``break``)."""
    resolution_cls = None

    @classmethod
    def fingerprint(cls, config):
        raise NotImplementedError

    @classmethod
    def detect(cls, old_config, new_config):
        if cls._differs(cls.fingerprint(old_config), cls.fingerprint(new_config), new_config):
            yield cls(old_config, new_config)

    @staticmethod
    def _differs(old, new, new_config):
        return old != new

    def marked_arguments(self, markers, conflicts):
        return {"change_type": markers.flag(self.resolution_cls.namespace())
                or A.CodeChange.BREAK}

    def _resolve(self, change_type=None):
        return self.resolution_cls(self, change_type)

    @property
    def diff(self):
        return colored_diff(pprint.pformat(self.fingerprint(self.old_config)),
                            pprint.pformat(self.fingerprint(self.new_config)))


@_register(50)
class CodeConflict(_TypedChangeConflict):
    """The user code's version-control state changed (only when the new run records one)."""
    resolution_cls = CodeResolution

    @classmethod
    def fingerprint(cls, config):
        return (config.get("metadata", {}) or {}).get("VCS")

    @staticmethod
    def _differs(old, new, new_config):
        return bool(new) and old != new

    def __repr__(self):
        old = pprint.pformat(self.fingerprint(self.old_config)).replace("\n", "")
        new = pprint.pformat(self.fingerprint(self.new_config)).replace("\n", "")
        return f"Old hash commit '{old}'  != new hash commit '{new}'"


@_register(60)
class CommandLineConflict(_TypedChangeConflict):
    """The non-prior arguments of the user's command line changed."""
    resolution_cls = CommandLineResolution

    @classmethod
    def fingerprint(cls, config):
        if not (config.get("metadata", {}) or {}).get("parser"):
            return ""
        parser = _user_parser(config)
        priors = parser.priors_to_normal()
        plain = sorted((k, a) for k, a in parser.parser.arguments.items() if k not in priors)
        return " ".join(f"{k} {a}" for k, a in plain)

    get_nameless_args = fingerprint

    @property
    def diff(self):
        return colored_diff(self.fingerprint(self.old_config), self.fingerprint(self.new_config))

    def __repr__(self):
        return (f"Old arguments '{self.fingerprint(self.old_config)}' != new arguments "
                f"'{self.fingerprint(self.new_config)}'")


@_register(70)
class ScriptConfigConflict(_TypedChangeConflict):
    """The non-prior content of the user script's configuration file changed."""
    resolution_cls = ScriptConfigResolution

    @classmethod
    def fingerprint(cls, config):
        if not (config.get("metadata", {}) or {}).get("parser"):
            return {}
        data = _user_parser(config).config_file_data
        if not isinstance(data, dict):
            return {}
        return {k: v for k, v in data.items()
                if not (isinstance(v, str) and v.startswith("orion~"))}

    get_nameless_config = fingerprint

    def __repr__(self):
        return "Script's configuration file changed"


# ---------------------------------------------------------------------------------- name
class ExperimentNameResolution(Resolution):
    """A new name (``--branch``, version 1), or the same name at the next version -- refused
    when the stored version already has children of that name (a new name is required)."""
    flag = "--branch"

    def __init__(self, conflict, new_name=None):
        super().__init__(conflict)
        old = conflict.old_config
        self.old_name = old["name"]
        self.old_version = old.get("version", 1)
        if new_name is not None and new_name != self.old_name:
            if _storage().fetch_experiments({"name": new_name,
                                             "metadata.user": conflict.username}):
                self._fail(f"Cannot branch from {self.old_name} with name {new_name} since "
                           "it already exists.")
            self.new_name, self.new_version = new_name, 1
        else:
            if _storage().fetch_experiments({"name": self.old_name,
                                             "refers.parent_id": old.get("_id")}):
                self._fail(f"Experiment name '{new_name}' already exist for user "
                           f"'{conflict.username}' and has children. Version cannot be "
                           "auto-incremented and a new name is required for branching.")
            self.new_name, self.new_version = self.old_name, self.old_version + 1
        conflict.new_config["name"] = self.new_name
        conflict.new_config["version"] = self.new_version

    def revert(self):
        self.conflict.new_config["name"] = self.old_name
        self.conflict.new_config["version"] = self.old_version
        return super().revert()

    @property
    def is_marked(self):
        return True

    def __repr__(self):
        return f"{self.flag} {self.new_name}"


@_register(0)
class ExperimentNameConflict(Conflict):
    @classmethod
    def detect(cls, old_config, new_config):
        yield cls(old_config, new_config)

    @property
    def username(self):
        return self.new_config["metadata"]["user"]

    def marked_arguments(self, markers, conflicts):
        name = markers.flag(ExperimentNameResolution.namespace())
        return {"new_name": name} if name else None

    def _resolve(self, new_name=None):
        return ExperimentNameResolution(self, new_name)

    def __repr__(self):
        return (f"Experiment name '{self.old_config['name']}' already exist for user "
                f"'{self.username}'")


# CLI flags of the resolutions (cli/evc.py builds the branching arguments from these)
FLAGS = {
    "branch": ExperimentNameResolution.flag,
    "algorithm": AlgorithmResolution.flag,
    "code": CodeResolution.flag,
    "cli": CommandLineResolution.flag,
    "config": ScriptConfigResolution.flag,
}
RESOLUTIONS = (ExperimentNameResolution, RemoveDimensionResolution, RenameDimensionResolution,
               AddDimensionResolution, ChangeDimensionResolution, AlgorithmResolution,
               CodeResolution, CommandLineResolution, ScriptConfigResolution)
