"""Gradient descent on the objective surface, driven by the ``gradient`` results a trial reports.

The reference ships this as an external plugin used to test entry-point discovery
(``tests/functional/gradient_descent_algo/src/orion/algo/gradient_descent.py:15-58``); it is a
built-in here (``requires='real'``), and tests/plugin_fixture registers a copy through an entry
point to exercise plugin discovery.
"""
from __future__ import annotations

import numpy

from .base import ALGORITHMS, BaseAlgorithm


@ALGORITHMS.register("gradient_descent")
class GradientDescent(BaseAlgorithm):
    """x <- x - learning_rate * grad; done once the step length is <= ``dx_tolerance``."""

    requires = "real"

    def __init__(self, space, learning_rate=1.0, dx_tolerance=1e-7):
        super().__init__(space, learning_rate=learning_rate, dx_tolerance=dx_tolerance)
        self.has_observed_once = False
        self.current_point = None
        self.gradient = numpy.array([numpy.inf])

    def suggest(self, num=1):
        if num != 1:
            raise ValueError("gradient descent suggests one point at a time")
        if not self.has_observed_once:
            return self.space.sample(1)
        self.current_point = self.current_point - self.learning_rate * self.gradient
        return [tuple(self.current_point)]

    def observe(self, points, results):
        self.current_point = numpy.asarray(points[-1], dtype=float)
        grad = results[-1].get("gradient")
        if grad is None:
            raise ValueError("gradient_descent needs trials to report a 'gradient' result")
        self.gradient = numpy.asarray(grad, dtype=float)
        self.has_observed_once = True

    @property
    def is_done(self):
        dx = self.learning_rate * numpy.sqrt(self.gradient.dot(self.gradient))
        return bool(dx <= self.dx_tolerance)

    @property
    def configuration(self):
        cfg = super().configuration
        return {"gradient_descent": cfg[type(self).__name__.lower()]}
