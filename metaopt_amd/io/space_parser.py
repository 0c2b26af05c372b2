"""Search-space priors in the user's command line and configuration file, and their per-trial
rendering (behaviour contract: reference ``src/orion/core/io/orion_cmdline_parser.py:31-456``).

* A command-line argument ``--lr~'loguniform(1e-5, 1)'`` declares the prior ``/lr``; ``-x~..``
  short options work too (``--x~..`` is read as ``-x``), and ``--out~/abs/path`` (a path or an
  empty value after ``~``) is an ordinary argument, not a prior.
* The argument named ``config_prefix`` (default ``config``) points at the user script's
  configuration file (YAML, JSON or any text file); every string leaf ``name~prior`` inside it
  declares the prior ``/a/b/c`` (its path in the document, list positions as numbers).
* ``format(config_path, trial, experiment)`` renders one trial: the configuration file with the
  trial's values in place of the priors, and the command line with the values substituted and
  ``{trial.xxx}`` / ``{exp.xxx}`` templates expanded.
* A prior declared both on the command line and in the file is an error.

Structure: :func:`_split_arg` turns one command-line word into the tokens the generic
:class:`CmdlineParser` sees; :func:`_leaves` is the single walker over the configuration
document, used both to collect the file's priors and to write a trial's values into a copy.
"""
from __future__ import annotations

import copy
import re
from collections import OrderedDict
from typing import Iterator, List, Tuple

from .cmdline_parser import CmdlineParser
from .convert import GenericConverter, infer_converter_from_file_type

PRIOR_TAG = "orion~"                       # how a command-line prior reaches CmdlineParser
_PRIOR = re.compile(r"(.+)~([\+\-\>]?.+)")  # "name~expression": group 2 = the prior


def _split_arg(arg: str) -> List[str]:
    """One command-line word -> the tokens handed to :class:`CmdlineParser`: ``--name~expr``
    becomes ``['--name', 'orion~expr']``; anything that is not an option carrying a prior stays
    a single token."""
    if not arg.startswith("-") or "~" not in arg:
        return [arg]
    name, expr = arg.split("~", 1)
    if expr == "" or expr.startswith("/"):         # '--path~/x': a value, not a prior
        return [arg]
    if len(name) == 3 and name.startswith("--"):    # '--x~' is the short option '-x'
        name = name[1:]
    return [name, PRIOR_TAG + expr]


def _leaves(node, path: str = "") -> Iterator[Tuple[str, object, object, object]]:
    """Depth-first ``(path, container, key, value)`` for every non-container leaf of a
    configuration document; ``container[key] = v`` replaces the leaf in place."""
    items = node.items() if isinstance(node, dict) else enumerate(node)
    for key, value in items:
        sub = f"{path}/{key}"
        if isinstance(value, (dict, list)):
            yield from _leaves(value, sub)
        else:
            yield sub, node, key, value


def _prior_of(value) -> str | None:
    """The prior expression of a ``name~expression`` string, else None."""
    if not isinstance(value, str):
        return None
    m = _PRIOR.match(value)
    return m.group(2) if m else None


class SpaceCmdlineParser:
    """Priors of a user command line (and its configuration file); renders trials back."""

    def __init__(self, config_prefix="config"):
        self.parser = CmdlineParser()
        self.config_prefix = config_prefix
        self.cmd_priors: "OrderedDict[str, str]" = OrderedDict()
        self.file_priors: "OrderedDict[str, str]" = OrderedDict()
        self.config_file_data = {}
        self.file_config_path = None
        self.converter = None

    # -- persisted state (stored with the experiment: the keys are a storage format) ---------
    def get_state_dict(self):
        return {"parser": self.parser.get_state_dict(),
                "cmd_priors": [[k, v] for k, v in self.cmd_priors.items()],
                "file_priors": [[k, v] for k, v in self.file_priors.items()],
                "config_file_data": self.config_file_data,
                "config_prefix": self.config_prefix,
                "file_config_path": self.file_config_path,
                "converter": None if self.converter is None else self.converter.get_state_dict()}

    def set_state_dict(self, state):
        self.parser.set_state_dict(state["parser"])
        self.cmd_priors = OrderedDict((k, v) for k, v in state["cmd_priors"])
        self.file_priors = OrderedDict((k, v) for k, v in state["file_priors"])
        self.config_file_data = state["config_file_data"]
        self.config_prefix = state["config_prefix"]
        self.file_config_path = state["file_config_path"]
        self.converter = None
        if self.file_config_path:
            self.converter = infer_converter_from_file_type(self.file_config_path)
            self.converter.set_state_dict(state["converter"])

    # -- parsing ------------------------------------------------------------------------------
    def parse(self, commandline):
        tokens = [tok for arg in commandline for tok in _split_arg(arg)]
        for key, value in self.parser.parse(tokens).items():
            if key == self.config_prefix:
                self._read_config_file(value)
                continue
            prior = _prior_of(value)
            if prior is not None:
                self.cmd_priors["/" + key.lstrip("/")] = prior
        both = set(self.cmd_priors) & set(self.file_priors)
        if both:
            raise ValueError(f"Prior(s) {sorted(both)} defined both on the command line and in "
                             "the configuration file")

    def _read_config_file(self, path):
        self.file_config_path = path
        self.converter = infer_converter_from_file_type(path)
        self.config_file_data = self.converter.parse(path)
        # the generic (text) converter hands out the bare expressions of its '~' markers
        bare = isinstance(self.converter, GenericConverter)
        doc = self.config_file_data
        if not isinstance(doc, (dict, list)):
            return
        for path_, _, _, value in _leaves(doc):
            if bare and isinstance(value, str):
                value = PRIOR_TAG + value
            prior = _prior_of(value)
            if prior is not None:
                self.file_priors[path_] = prior

    @property
    def priors(self) -> OrderedDict:
        out = OrderedDict(self.file_priors)
        out.update(self.cmd_priors)
        return out

    def priors_to_normal(self):
        return {k.lstrip("/"): v for k, v in self.cmd_priors.items()}

    # -- rendering ----------------------------------------------------------------------------
    def format(self, config_path=None, trial=None, experiment=None):
        if self.file_config_path:
            if config_path is None:
                raise ValueError("this command line reads a configuration file: rendering a "
                                 "trial needs `config_path` for its instance")
            self._write_config_instance(config_path, trial)
        args = copy.deepcopy(self.parser.arguments)
        for param in (trial.params if trial is not None else ()):
            args[param.name.lstrip("/")] = param.value
        if config_path is not None:
            args[self.config_prefix] = config_path
        context = {"trial": trial, "exp": experiment}
        return [word.format(**context) for word in self.parser.format(args)]

    def _write_config_instance(self, config_path, trial):
        doc = copy.deepcopy(self.config_file_data)
        values = {p.name: p.value for p in (trial.params if trial is not None else ())
                  if p.name in self.file_priors}
        if values and isinstance(doc, (dict, list)):
            for path_, container, key, _ in list(_leaves(doc)):
                if path_ in values:
                    container[key] = values[path_]
        self.converter.generate(config_path, doc)


OrionCmdlineParser = SpaceCmdlineParser  # reference-compatible name
