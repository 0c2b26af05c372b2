"""User-script configuration file converters (reference: ``src/orion/core/io/convert.py:31-285``).

``YAMLConverter`` (.yml/.yaml), ``JSONConverter`` (.json) and ``GenericConverter`` (any text file:
``name~prior(...)`` expressions are located by regex, replaced by ``{name!s}`` placeholders, and the
file is re-rendered per trial with the sampled values).
"""
from __future__ import annotations

import json
import os
import re
from collections import defaultdict, deque

import yaml


class BaseConverter:
    file_extensions: list = []

    def get_state_dict(self):
        return {}

    def set_state_dict(self, state):
        pass

    def parse(self, filepath):
        raise NotImplementedError

    def generate(self, filepath, data):
        raise NotImplementedError


class YAMLConverter(BaseConverter):
    file_extensions = [".yml", ".yaml"]

    def parse(self, filepath):
        with open(filepath) as f:
            return yaml.safe_load(f)

    def generate(self, filepath, data):
        with open(filepath, "w") as f:
            yaml.safe_dump(data, f, default_flow_style=False)


class JSONConverter(BaseConverter):
    file_extensions = [".json"]

    def parse(self, filepath):
        with open(filepath) as f:
            return json.load(f)

    def generate(self, filepath, data):
        with open(filepath, "w") as f:
            json.dump(data, f)


def _nesteddict():
    return defaultdict(_nesteddict)


class GenericConverter(BaseConverter):
    """Templating converter for arbitrary text configuration files."""

    DEFAULT_REGEX = r"([\/]?[\w|\/|-]+)~([\+]?.*\)|\-|\>[A-Za-z_]\w*)"

    def __init__(self, regex=DEFAULT_REGEX, expression_prefix=""):
        self.regex = re.compile(regex)
        self.expression_prefix = expression_prefix
        self.template = None
        self.has_leading = {}

    def get_state_dict(self):
        return dict(regex=self.regex.pattern, expression_prefix=self.expression_prefix,
                    template=self.template, has_leading=self.has_leading)

    def set_state_dict(self, state):
        self.regex = re.compile(state["regex"])
        self.expression_prefix = state["expression_prefix"]
        self.template = state["template"]
        self.has_leading = state["has_leading"]

    def _conflict(self, path, namespace):
        raise ValueError(f"Namespace conflict in configuration file '{path}', under '{namespace}'")

    def parse(self, filepath):
        with open(filepath) as f:
            text = f.read()
        pairs = self.regex.findall(text)
        found = dict(pairs)
        if len(pairs) != len(found):
            names = [p[0] for p in pairs]
            for n in names:
                if names.count(n) != 1:
                    self._conflict(filepath, n)
        escaped = text.replace("{", "{{").replace("}", "}}")
        self.template, nsubs = self.regex.subn(r"{\1!s}", escaped)
        if nsubs != len(found):  # pragma: no cover - regex bug guard
            raise RuntimeError("inconsistent generic-converter substitution")
        nested = _nesteddict()
        for namespace, expression in found.items():
            keys = namespace.split("/")
            if not keys[0]:
                keys = keys[1:]
                self.has_leading[namespace[1:]] = "/"
            cur = nested
            for i, k in enumerate(keys[:-1]):
                cur = cur[k]
                if isinstance(cur, str):
                    self._conflict(filepath, "/".join(keys[:i + 1]))
            if cur[keys[-1]]:
                self._conflict(filepath, namespace)
            cur[keys[-1]] = self.expression_prefix + expression
        return _to_dict(nested)

    def generate(self, filepath, data):
        flat = {}
        stack = deque([([], data)])
        while stack:
            namespace, stuff = stack.pop()
            if isinstance(stuff, dict):
                for k, v in stuff.items():
                    stack.append((["/".join(namespace + [str(k)])], v))
            else:
                name = namespace[0]
                flat[self.has_leading.get(name, "") + name] = stuff
        doc = self.template.format(**flat)
        with open(filepath, "w") as f:
            f.write(doc)


def _to_dict(d):
    if isinstance(d, defaultdict):
        return {k: _to_dict(v) for k, v in d.items()}
    return d


CONVERTERS = [YAMLConverter, JSONConverter]


def infer_converter_from_file_type(config_path, regex=None, default_keyword=""):
    _, ext = os.path.splitext(os.path.abspath(config_path))
    for klass in CONVERTERS:
        if ext in klass.file_extensions:
            return klass()
    if regex is None:
        return GenericConverter(expression_prefix=default_keyword)
    return GenericConverter(regex, expression_prefix=default_keyword)
