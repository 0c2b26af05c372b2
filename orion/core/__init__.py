"""``orion.core``: the configuration object, re-exported from :mod:`metaopt_amd.core.config`."""
from metaopt_amd.core.config import config  # noqa: F401
