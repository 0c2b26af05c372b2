"""The prior DSL: ``name~'loguniform(1e-5, 1.0)'`` -> :class:`~metaopt_amd.space.dims.Dimension`.

Grammar and aliases follow the reference (``src/orion/core/io/space_builder.py:89-332``):

* ``choices([...])`` / ``choices({cat: prob})`` / ``choices(a, b, c)``  -> Categorical
* ``fidelity(low, high, base=2)``                                      -> Fidelity
* ``uniform(a, b)`` means U[a, b) (NOT scipy's loc/scale convention)   -> Real / Integer
* ``normal`` / ``gaussian`` -> scipy ``norm``; ``loguniform`` -> scipy ``reciprocal``
* any other ``scipy.stats`` continuous distribution -> Real (Integer with ``discrete=True``),
  any discrete one -> Integer
* dimension kwargs: ``discrete``, ``default_value``, ``shape``, ``low``, ``high``
* EVC markers: expressions starting with ``-`` or ``>`` are not built, a leading ``+`` is stripped.

Unlike the reference's restricted ``eval``, expressions are parsed with :mod:`ast` and only
literals (numbers, strings, lists, tuples, dicts, ``inf``/``nan``, unary minus) are accepted as
arguments, so a prior string can never execute code.
"""
from __future__ import annotations

import ast
import math
import re
from collections import OrderedDict
from typing import Dict, Tuple

from scipy.stats import distributions as sp_dists

from .dims import Categorical, Dimension, Fidelity, Integer, Real, Space

_CALL_RE = re.compile(r"^\s*([A-Za-z_][A-Za-z0-9_]*)\s*\((.*)\)\s*$", re.S)
_NAMED_CONSTANTS = {"inf": math.inf, "nan": math.nan, "True": True, "False": False, "None": None}


class PriorSyntaxError(TypeError):
    pass


def _literal(node):
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.Name) and node.id in _NAMED_CONSTANTS:
        return _NAMED_CONSTANTS[node.id]
    if isinstance(node, ast.Attribute) and node.attr in ("inf", "nan") and \
            isinstance(node.value, ast.Name) and node.value.id in ("numpy", "np", "math"):
        return _NAMED_CONSTANTS[node.attr]
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, (ast.USub, ast.UAdd)):
        v = _literal(node.operand)
        return -v if isinstance(node.op, ast.USub) else +v
    if isinstance(node, ast.BinOp) and isinstance(node.op, (ast.Add, ast.Sub, ast.Mult, ast.Div,
                                                            ast.Pow)):
        a, b = _literal(node.left), _literal(node.right)
        if not all(isinstance(v, (int, float)) for v in (a, b)):
            raise PriorSyntaxError("arithmetic only on numbers")
        return {ast.Add: lambda: a + b, ast.Sub: lambda: a - b, ast.Mult: lambda: a * b,
                ast.Div: lambda: a / b, ast.Pow: lambda: a ** b}[type(node.op)]()
    if isinstance(node, ast.List):
        return [_literal(e) for e in node.elts]
    if isinstance(node, ast.Tuple):
        return tuple(_literal(e) for e in node.elts)
    if isinstance(node, ast.Dict):
        return {_literal(k): _literal(v) for k, v in zip(node.keys, node.values)}
    raise PriorSyntaxError(f"unsupported expression in prior arguments: {ast.dump(node)}")


def parse_prior(expression: str) -> Tuple[str, tuple, dict]:
    """``'uniform(-3, 5, shape=2)'`` -> ``('uniform', (-3, 5), {'shape': 2})`` (literals only)."""
    if "__" in expression or ";" in expression:
        raise RuntimeError("Cannot use builtins, '__' or ';'. Sorry.")
    m = _CALL_RE.match(expression)
    if not m:
        raise PriorSyntaxError(f"Please provide a valid form for prior: "
                               f"'distribution(*args, **kwargs)'\nProvided: '{expression}'")
    try:
        tree = ast.parse(expression.strip(), mode="eval")
    except SyntaxError as exc:
        raise PriorSyntaxError(f"cannot parse prior '{expression}': {exc}") from exc
    call = tree.body
    if not isinstance(call, ast.Call) or not isinstance(call.func, ast.Name):
        raise PriorSyntaxError(f"prior must be a call 'distribution(...)', got '{expression}'")
    args = tuple(_literal(a) for a in call.args)
    kwargs = {kw.arg: _literal(kw.value) for kw in call.keywords}
    return call.func.id, args, kwargs


def _real_or_int(kwargs):
    return Integer if kwargs.pop("discrete", False) else Real


class DimensionBuilder:
    """Build a :class:`Dimension` from a name and a prior expression."""

    def __init__(self):
        self.name = None

    # -- aliases -----------------------------------------------------------------------------
    def choices(self, *args, **kwargs):
        if not args:
            raise TypeError(f"Parameter '{self.name}': Expected argument with categories.")
        if isinstance(args[0], (dict, list)):
            return Categorical(self.name, *args, **kwargs)
        return Categorical(self.name, args, **kwargs)

    def fidelity(self, *args, **kwargs):
        return Fidelity(self.name, *args, **kwargs)

    def uniform(self, *args, **kwargs):
        klass = _real_or_int(kwargs)
        if len(args) == 2:
            return klass(self.name, "uniform", args[0], args[1] - args[0], **kwargs)
        return klass(self.name, "uniform", *args, **kwargs)

    def gaussian(self, *args, **kwargs):
        return self.normal(*args, **kwargs)

    def normal(self, *args, **kwargs):
        klass = _real_or_int(kwargs)
        return klass(self.name, "norm", *args, **kwargs)

    def loguniform(self, *args, **kwargs):
        klass = _real_or_int(kwargs)
        return klass(self.name, "reciprocal", *args, **kwargs)

    _ALIASES = ("choices", "fidelity", "uniform", "gaussian", "normal", "loguniform")

    def _build(self, name: str, expression: str) -> Dimension:
        self.name = name
        prior, args, kwargs = parse_prior(expression)
        if prior in self._ALIASES:
            return getattr(self, prior)(*args, **kwargs)
        if hasattr(sp_dists._continuous_distns, prior):  # scipy's public registry modules
            klass = _real_or_int(kwargs)
        elif hasattr(sp_dists._discrete_distns, prior):
            klass = Integer
        else:
            raise TypeError(f"Parameter '{name}': '{prior}' does not correspond to a supported "
                            "distribution.")
        return klass(name, prior, *args, **kwargs)

    def build(self, name: str, expression: str) -> Dimension:
        """Build and warm up (one sample) so a bad prior fails at definition time."""
        try:
            dim = self._build(name, expression)
        except PriorSyntaxError as exc:
            raise TypeError(f"Parameter '{name}': {exc}") from exc
        except ValueError as exc:
            raise TypeError(f"Parameter '{name}': Incorrect arguments.") from exc
        try:
            dim.sample()
        except TypeError as exc:
            raise TypeError(f"Parameter '{name}': Incorrect arguments for distribution "
                            f"'{dim.prior_name}'.") from exc
        except ValueError as exc:
            raise TypeError(f"Parameter '{name}': Incorrect arguments.") from exc
        return dim


def should_not_be_built(expression: str) -> bool:
    return expression.startswith("-") or expression.startswith(">")


def remove_marker(expression: str, marker: str = "+") -> str:
    return expression.replace(marker, "", 1) if expression.startswith(marker) else expression


class SpaceBuilder:
    """Build a :class:`Space` from ``{name: prior_expression}`` (EVC markers honoured)."""

    def __init__(self):
        self.dimbuilder = DimensionBuilder()
        self.space = None

    def build(self, configuration: Dict[str, str]) -> Space:
        self.space = Space()
        for name, expression in configuration.items():
            if should_not_be_built(expression):
                continue
            expression = remove_marker(expression)
            dim = self.dimbuilder.build(name, expression)
            try:
                self.space.register(dim)
            except ValueError as exc:
                raise ValueError(f"Conflict for name '{name}' in parameters") from exc
        return self.space


def build_space(priors: Dict[str, str]) -> Space:
    """Convenience: ``build_space({'lr': 'loguniform(1e-4, 1)'})``."""
    return SpaceBuilder().build(OrderedDict(priors))
