"""Generic command-line parsing and templating.

Same contract as the reference's ``CmdlineParser`` (``src/orion/core/io/cmdline_parser.py``):

* ``parse(argv)`` returns an ordered ``{key: value}``: leading positionals become ``_pos_N``
  (``N`` counts the keys before them), ``--a=b`` / ``--a b`` / ``-a b`` a value, a bare option
  ``True``, an option followed by several words a list; words naming existing paths are made
  absolute;
* ``template`` is the command line as format strings (``"--lr"``, ``"{lr}"``, ``"{x[1]}"``,
  ``"{_pos_0}"``) and ``format(config)`` re-renders it with new values;
* ``get_state_dict`` / ``set_state_dict`` round-trip ``{arguments: [[k, v]...], template}``
  through an experiment's ``metadata.parser`` (format kept for stored experiments).

Implementation: argv is first cut into *groups* (an option word and the words up to the next
option, or one positional); keys, values and template pieces are then derived per group.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Iterator, List, Tuple


def _groups(argv) -> Iterator[Tuple[bool, str, List[str]]]:
    """(is_option, name or positional word, words) for each group of ``argv``."""
    current = None
    for word in argv:
        if word.startswith("-"):
            if current is not None:
                yield current
            name, eq, inline = word.lstrip("-").partition("=")
            current = (True, name, [inline] if eq else [])
        elif current is not None:
            if word.strip(" "):
                current[2].append(word)
        else:
            yield (False, word, [])
    if current is not None:
        yield current


def _absolute(value):
    if isinstance(value, list):
        return [_absolute(v) for v in value]
    if isinstance(value, str) and os.path.exists(value):
        return os.path.abspath(value)
    return value


def _option(key: str) -> str:
    return ("--" if len(key) > 1 else "-") + key


class CmdlineParser:
    def __init__(self):
        self.arguments: "OrderedDict[str, object]" = OrderedDict()
        self.template: List[str] = []
        self._already_parsed = False

    # -- persistence ------------------------------------------------------------------------------
    def get_state_dict(self):
        return {"arguments": [[k, v] for k, v in self.arguments.items()],
                "template": list(self.template)}

    def set_state_dict(self, state):
        self.arguments = OrderedDict((k, v) for k, v in state["arguments"])
        self.template = list(state["template"])
        self._already_parsed = bool(self.template)

    # -- rendering --------------------------------------------------------------------------------
    def format(self, configuration):
        """The command line with ``configuration``'s values substituted."""
        return [piece if piece.startswith("-") else piece.format(**configuration)
                for piece in self.template]

    # -- parsing ----------------------------------------------------------------------------------
    def parse(self, commandline):
        if self._already_parsed:
            raise RuntimeError("The commandline has already been parsed.")
        arguments: "OrderedDict[str, object]" = OrderedDict()
        template: List[str] = []
        for is_option, name, words in _groups(commandline):
            if not is_option:
                key = f"_pos_{len(arguments)}"
                arguments[key] = _absolute(name)
                template.append("{" + key + "}")
                continue
            if name in arguments:
                raise ValueError(f"Conflict: argument '{name}' appears twice on the command line")
            value = True if not words else (words[0] if len(words) == 1 else list(words))
            arguments[name] = _absolute(value)
            template.append(_option(name))
            if isinstance(value, list):
                template.extend("{%s[%d]}" % (name, i) for i in range(len(value)))
            elif value is not True:
                template.append("{" + name + "}")
        self.arguments = arguments
        self.template = template
        self._already_parsed = True
        return self.arguments
