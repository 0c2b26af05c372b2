"""Oríon compatibility surface of ``metaopt_amd``.

Existing Oríon user scripts and plugins keep their imports: ``from orion.client import
report_results`` (reference ``src/orion/client/__init__.py:25-48``), the ``orion`` console
command (``orion.core.cli:main``, reference ``setup.py:39-42``) and the plugin base classes
(``orion.algo.base.BaseAlgorithm``, ``orion.algo.space``).  Every name here is the
``metaopt_amd`` object itself, re-exported; nothing is re-implemented.
"""
from metaopt_amd import __version__  # noqa: F401
