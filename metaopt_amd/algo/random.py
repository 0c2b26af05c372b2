"""Random search (reference: ``src/orion/algo/random.py:16-65``)."""
from __future__ import annotations

import numpy

from .base import ALGORITHMS, BaseAlgorithm


@ALGORITHMS.register()
class Random(BaseAlgorithm):
    """Sample points from the space's priors; observations are ignored."""

    trusted_suggestions = True

    def __init__(self, space, seed=None):
        super().__init__(space, seed=seed)

    def seed_rng(self, seed):
        self.rng = numpy.random.RandomState(seed)

    @property
    def state_dict(self):
        return {"rng_state": self.rng.get_state()}

    def set_state(self, state_dict):
        self.seed_rng(0)
        self.rng.set_state(state_dict["rng_state"])

    def suggest(self, num=1):
        return self.space.sample(num, seed=tuple(self.rng.randint(0, 1000000, size=3)))

    def observe(self, points, results):
        pass
