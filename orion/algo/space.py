"""``orion.algo.space``: search-space dimensions (:mod:`metaopt_amd.space.dims`)."""
from metaopt_amd.space.dims import (Categorical, Dimension, Fidelity, Integer, Real,  # noqa: F401
                                    Space, check_random_state)
