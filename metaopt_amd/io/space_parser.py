"""Prior extraction from the user's command line and configuration file, and per-trial
re-rendering of both (reference: ``src/orion/core/io/orion_cmdline_parser.py:31-456``).

* ``--lr~'loguniform(1e-5, 1)'`` on the command line is rewritten to ``--lr orion~loguniform(..)``
  and recorded as prior ``/lr``; ``-x~...`` short options are supported, ``--path~/abs`` is not a
  prior;
* the argument named ``config_prefix`` (default ``config``) names the user-script configuration
  file (YAML, JSON or any text file); priors inside it become ``/a/b/c`` (nested namespace);
* ``format(config_path, trial, experiment)`` writes the per-trial configuration file, substitutes
  the trial's values into the command line and expands ``{trial.xxx}`` / ``{exp.xxx}`` templates
  (e.g. ``--checkpoint {trial.working_dir}/model.pt``).
Duplicate priors between the command line and the file raise ``ValueError``.
"""
from __future__ import annotations

import copy
import re
from collections import OrderedDict

from .cmdline_parser import CmdlineParser
from .convert import GenericConverter, infer_converter_from_file_type

PRIOR_TAG = "orion~"


def _is_nonprior_wave(arg: str) -> bool:
    return arg.startswith("/") or arg == ""


class SpaceCmdlineParser:
    """Parse the user command line for priors and render it back for a trial."""

    def __init__(self, config_prefix="config"):
        self.parser = CmdlineParser()
        self.cmd_priors = OrderedDict()
        self.file_priors = OrderedDict()
        self.config_file_data = {}
        self.config_prefix = config_prefix
        self.file_config_path = None
        self.converter = None
        self.prior_regex = re.compile(r"(.+)~([\+\-\>]?.+)")

    # -- state -------------------------------------------------------------------------------
    def get_state_dict(self):
        return dict(parser=self.parser.get_state_dict(),
                    cmd_priors=[list(x) for x in self.cmd_priors.items()],
                    file_priors=[list(x) for x in self.file_priors.items()],
                    config_file_data=self.config_file_data,
                    config_prefix=self.config_prefix,
                    file_config_path=self.file_config_path,
                    converter=self.converter.get_state_dict() if self.converter else None)

    def set_state_dict(self, state):
        self.parser.set_state_dict(state["parser"])
        self.cmd_priors = OrderedDict(state["cmd_priors"])
        self.file_priors = OrderedDict(state["file_priors"])
        self.config_file_data = state["config_file_data"]
        self.config_prefix = state["config_prefix"]
        self.file_config_path = state["file_config_path"]
        if self.file_config_path:
            self.converter = infer_converter_from_file_type(self.file_config_path)
            self.converter.set_state_dict(state["converter"])

    # -- parsing -----------------------------------------------------------------------------
    def parse(self, commandline):
        configuration = self.parser.parse(self._replace_priors(commandline))
        for key, value in configuration.items():
            if key == self.config_prefix:
                self.file_config_path = value
                self._load_config(value)
            else:
                self._extract_prior(key, value, self.cmd_priors)
        dup = set(self.cmd_priors) & set(self.file_priors)
        if dup:
            raise ValueError(f"Conflict: definition of same prior in commandline and config: {dup}")

    @property
    def priors(self) -> OrderedDict:
        p = copy.deepcopy(self.file_priors)
        p.update(self.cmd_priors)
        return p

    @staticmethod
    def _replace_priors(args):
        out = []
        for item in args:
            if item.startswith("-"):
                parts = item.split("~")
                if len(parts) > 1 and _is_nonprior_wave(parts[1]):
                    out.append(item)
                    continue
                if parts[0].startswith("--") and len(parts[0]) == 3:
                    parts[0] = parts[0][1:]
                out.append(parts[0])
                if len(parts) > 1:
                    out.append(PRIOR_TAG + "~".join(parts[1:]))
            else:
                out.append(item)
        return out

    def _load_config(self, path):
        self.converter = infer_converter_from_file_type(path)
        self.config_file_data = self.converter.parse(path)
        generic = isinstance(self.converter, GenericConverter)
        self._extract(self.config_file_data, "", generic)

    def _extract(self, value, depth, generic=False):
        if isinstance(value, dict):
            for k, v in value.items():
                self._extract(v, f"{depth}/{k}", generic)
        elif isinstance(value, list):
            for i, v in enumerate(value):
                self._extract(v, f"{depth}/{i}", generic)
        elif isinstance(value, str):
            if generic:  # the generic converter yields bare expressions (no 'name~' prefix)
                value = PRIOR_TAG + value
            if "~" in value:
                self._extract_prior(depth, value, self.file_priors)

    def _extract_prior(self, key, value, insert_into):
        if not isinstance(value, str):
            return
        m = self.prior_regex.match(value)
        if m is None:
            return
        name = key if key.startswith("/") else "/" + key
        insert_into[name] = m.group(2)

    # -- rendering ---------------------------------------------------------------------------
    def format(self, config_path=None, trial=None, experiment=None):
        if self.file_config_path and config_path is None:
            raise ValueError("The configuration contains a config file. Cannot format without a "
                             "`config_path` argument.")
        if self.file_config_path:
            self._create_config_file(config_path, trial)
        configuration = self._build_configuration(trial)
        if config_path is not None:
            configuration[self.config_prefix] = config_path
        templated = self.parser.format(configuration)
        ctx = dict(trial=trial, exp=experiment)
        return [item.format(**ctx) for item in templated]

    def _create_config_file(self, config_path, trial):
        instance = copy.deepcopy(self.config_file_data)
        for param in trial.params:
            if param.name not in self.file_priors:
                continue
            cur = instance
            for key in param.name.split("/")[1:]:
                if isinstance(cur, list):
                    if not key.isdigit():
                        continue
                    key = int(key)
                    if key >= len(cur):
                        break
                if isinstance(cur[key], str):
                    cur[key] = param.value
                else:
                    cur = cur[key]
        self.converter.generate(config_path, instance)

    def _build_configuration(self, trial):
        configuration = copy.deepcopy(self.parser.arguments)
        if trial is not None:
            for param in trial.params:
                configuration[param.name.lstrip("/")] = param.value
        return configuration

    def priors_to_normal(self):
        return {k.lstrip("/"): v for k, v in self.cmd_priors.items()}


OrionCmdlineParser = SpaceCmdlineParser  # reference-compatible name
