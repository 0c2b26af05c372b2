"""``orion.core.cli``: the command line (``orion hunt ...``), i.e. :func:`metaopt_amd.cli.main`."""
from metaopt_amd.cli import main  # noqa: F401
