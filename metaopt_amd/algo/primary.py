"""Wrapper that adapts the user's space to an algorithm's requirements
(reference: ``src/orion/core/worker/primary_algo.py:17-144``).

Suggested points are checked against the transformed space and reversed to the user's space;
observed points are checked against the user's space and transformed forward.
"""
from __future__ import annotations

import numpy

from ..space.transformer import build_required_space
from .base import BaseAlgorithm, create_algo


def _plain(v):
    if isinstance(v, numpy.ndarray) and v.shape == ():
        return v.item()
    if isinstance(v, numpy.generic):
        return v.item()
    return v


class PrimaryAlgo(BaseAlgorithm):
    def __init__(self, space, algorithm_config):
        self._space = space
        self._param_names = ["algorithm"]
        self.algorithm = create_algo(space, algorithm_config)
        self.transformed_space = build_required_space(self.algorithm.requires, space)
        self.algorithm.space = self.transformed_space

    def seed_rng(self, seed):
        self.algorithm.seed_rng(seed)

    @property
    def state_dict(self):
        return self.algorithm.state_dict

    def set_state(self, state_dict):
        self.algorithm.set_state(state_dict)

    def full_state(self):
        return self.algorithm.full_state()

    def suggest(self, num=1):
        points = self.algorithm.suggest(num)
        if points is None:
            return None
        check = not getattr(self.algorithm, "trusted_suggestions", False)
        if not check and self.transformed_space._is_identity():
            # draws of space.sample (python scalars) or earlier points: nothing to convert
            return [p if type(p) is tuple else tuple(p) for p in points]
        out = []
        for p in points:
            if check and p not in self.transformed_space:
                raise ValueError(f"Point is not contained in space:\nPoint: {p}\n"
                                 f"Space: {self.transformed_space}")
            out.append(tuple(_plain(v) for v in self.transformed_space.reverse(p)))
        return out

    def observe(self, points, results, check=True):
        """``check=False``: the caller vouches that the points came from :meth:`suggest` (which
        validated them) -- the device sweep observes thousands of points per sync."""
        if len(points) != len(results):
            raise ValueError("points and results differ in length")
        if not check and self.transformed_space._is_identity():
            self.algorithm.observe(points, results)
            return
        tpoints = []
        for p in points:
            if check and p not in self.space:
                raise ValueError(f"Point {p} is not contained in space {self.space}")
            tpoints.append(self.transformed_space.transform(p))
        self.algorithm.observe(tpoints, results)

    def observe_objectives(self, points, objectives, ids=None):
        """:meth:`observe` of suggested points (``check=False``) with bare objective values --
        the device sweep's path: no result dict per point when the algorithm takes floats.
        ``ids``: the algorithm's own ids of the points (``get_id``), when the caller has them."""
        inner = getattr(self.algorithm, "observe_objectives", None)
        if inner is None or not self.transformed_space._is_identity():
            self.observe(points, [{"objective": o, "constraint": [], "gradient": None}
                                  for o in objectives], check=False)
            return
        if ids is not None:
            inner(points, objectives, ids=ids)
        else:
            inner(points, objectives)

    def parent_of(self, point):
        """Point whose trained state ``point`` resumes from (PBT exploit, ASHA promotion), if the
        algorithm tracks lineage; None otherwise."""
        fn = getattr(self.algorithm, "parent_of", None)
        if fn is None:
            return None
        parent = fn(self.transformed_space.transform(point))
        if parent is None:
            return None
        return tuple(_plain(v) for v in self.transformed_space.reverse(parent))

    @property
    def is_done(self):
        return self.algorithm.is_done

    @property
    def synchronous(self):
        return bool(getattr(self.algorithm, "synchronous", False))

    def score(self, point):
        return self.algorithm.score(self.transformed_space.transform(point))

    def judge(self, point, measurements):
        return self.algorithm.judge(self.transformed_space.transform(point), measurements)

    @property
    def should_suspend(self):
        return self.algorithm.should_suspend

    @property
    def configuration(self):
        return self.algorithm.configuration

    @property
    def space(self):
        return self._space
