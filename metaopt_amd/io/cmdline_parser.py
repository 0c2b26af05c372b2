"""Generic command-line parsing and templating (reference:
``src/orion/core/io/cmdline_parser.py:22-265``).

``parse(argv)`` maps positionals to ``_pos_N``, ``--a=b``/``--a b`` to values, bare flags to
``True`` and multi-valued options to lists (existing paths become absolute), and builds a
``template`` that ``format(configuration)`` re-renders.  ``get_state_dict``/``set_state_dict``
round-trip through the experiment's ``metadata.parser``.
"""
from __future__ import annotations

import os
from collections import OrderedDict


class CmdlineParser:
    def __init__(self):
        self.arguments = OrderedDict()
        self._already_parsed = False
        self.template = []

    def get_state_dict(self):
        return dict(arguments=[list(x) for x in self.arguments.items()], template=list(self.template))

    def set_state_dict(self, state):
        self.arguments = OrderedDict(state["arguments"])
        self.template = list(state["template"])
        self._already_parsed = bool(self.template)

    def format(self, configuration):
        out = []
        for item in self.template:
            out.append(item if item.startswith("-") else item.format(**configuration))
        return out

    def parse(self, commandline):
        if self._already_parsed:
            raise RuntimeError("The commandline has already been parsed.")
        self.arguments = self._parse_arguments(commandline)
        for key, value in self.arguments.items():
            if key.startswith("_"):
                self.template.append("{" + key + "}")
                continue
            arg = self._key_to_arg(key)
            if arg in self.template:
                continue
            self.template.append(arg)
            if isinstance(value, bool):
                continue
            if not isinstance(value, list):
                self.template.append("{" + key + "}")
                continue
            for pos in range(len(value)):
                self.template.append("{" + key + "[" + str(pos) + "]}")
        self._already_parsed = True
        return self.arguments

    @staticmethod
    def _key_to_arg(key):
        return "--" + key if len(key) > 1 else "-" + key

    def _parse_arguments(self, commandline):
        args = OrderedDict()
        name = None
        for item in commandline:
            if item.startswith("-"):
                name = item.lstrip("-")
                parts = name.split("=")
                name = parts[0]
                if name in args:
                    raise ValueError(f"Conflict: two arguments have the same name: {name}")
                args[name] = []
                if len(parts) > 1:
                    args[name].append(parts[-1])
            elif name is not None and item.strip(" "):
                args[name].append(item)
            elif name is None:
                args[f"_pos_{len(args)}"] = item
        for key, value in args.items():
            if isinstance(value, list):
                if not value:
                    value = True
                elif len(value) == 1:
                    value = value[0]
            args[key] = self._parse_paths(value)
        return args

    def _parse_paths(self, value):
        if isinstance(value, list):
            return [self._parse_paths(v) for v in value]
        if isinstance(value, str) and os.path.exists(value):
            return os.path.abspath(value)
        return value
