"""Exhaustive grid search over a space (not in the reference; Oríon later added one).

Every dimension contributes a list of values: all categories of a categorical, the maximum of a
fidelity, ``n_values`` evenly spaced values of a real (geometrically spaced for log priors) and
up to ``n_values`` distinct integers of an integer dimension.  Points are the Cartesian product,
visited in a fixed order; ``is_done`` once all are suggested and observed.
"""
from __future__ import annotations

import itertools

import numpy

from .base import ALGORITHMS, BaseAlgorithm


def _grid_values(dim, n):
    if dim.type == "categorical":
        return list(dim.categories)
    if dim.type == "fidelity":
        return [dim.high]
    if getattr(dim, "shape", ()):
        raise ValueError(f"grid search does not support shaped dimension {dim.name}")
    low, high = dim.interval()
    if not (numpy.isfinite(low) and numpy.isfinite(high)):
        low, high = dim.interval(0.95)
    log = getattr(dim, "prior_name", "") == "reciprocal" and low > 0
    if dim.type == "integer":
        hi = high - 1
        if log:
            vals = numpy.geomspace(max(low, 1), hi, n)
        else:
            vals = numpy.linspace(low, hi, n)
        return sorted(set(int(round(v)) for v in vals))
    hi = numpy.nextafter(high, -numpy.inf)
    vals = numpy.geomspace(low, hi, n) if log else numpy.linspace(low, hi, n)
    return [float(v) for v in vals]


@ALGORITHMS.register()
class GridSearch(BaseAlgorithm):
    def __init__(self, space, n_values=10, seed=None):
        super().__init__(space, n_values=n_values, seed=seed)
        self._grid = None
        self._next = 0
        self._observed = set()

    def _build(self):
        n = self.n_values
        per_dim = []
        for dim in self.space.values():
            k = n.get(dim.name, 10) if isinstance(n, dict) else n
            per_dim.append(_grid_values(dim, int(k)))
        self._grid = [tuple(p) for p in itertools.product(*per_dim)]

    @property
    def grid(self):
        if self._grid is None:
            self._build()
        return self._grid

    @property
    def state_dict(self):
        return {"next": self._next}

    def set_state(self, state_dict):
        self._next = state_dict.get("next", 0)

    def suggest(self, num=1):
        pts = self.grid[self._next:self._next + num]
        self._next += len(pts)
        return pts or None

    def observe(self, points, results):
        for p in points:
            self._observed.add(tuple(p))

    @property
    def is_done(self):
        return self._next >= len(self.grid) and len(self._observed) >= len(self.grid)
