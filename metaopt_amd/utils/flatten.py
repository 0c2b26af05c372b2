"""Nested dict <-> dotted-key dict (reference: ``src/orion/core/utils/flatten.py:16-51``)."""
from __future__ import annotations


def flatten(dictionary: dict, sep: str = ".") -> dict:
    """``{'a': {'b': 1}}`` -> ``{'a.b': 1}`` (empty sub-dicts are kept as values)."""
    out = {}

    def _rec(prefix, d):
        for k, v in d.items():
            key = f"{prefix}{sep}{k}" if prefix else str(k)
            if isinstance(v, dict) and v:
                _rec(key, v)
            else:
                out[key] = v

    _rec("", dictionary)
    return out


def unflatten(dictionary: dict, sep: str = ".") -> dict:
    """``{'a.b': 1}`` -> ``{'a': {'b': 1}}``."""
    out: dict = {}
    for key, value in dictionary.items():
        parts = key.split(sep)
        d = out
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = value
    return out
