"""``orion.algo.base``: :class:`BaseAlgorithm` and the algorithm registry of metaopt_amd."""
from metaopt_amd.algo.base import ALGORITHMS, BaseAlgorithm  # noqa: F401

OptimizationAlgorithm = ALGORITHMS
