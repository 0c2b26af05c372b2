"""Per-trial working directories (reference: ``src/orion/core/utils/working_dir.py:15-49``)."""
from __future__ import annotations

import os
import shutil
import tempfile


class WorkingDir:
    """Context manager: a temporary directory (removed on exit) or a persistent
    ``<working_dir>/<prefix><suffix>`` directory when ``temp=False``."""

    def __init__(self, working_dir, temp=True, suffix=None, prefix=None):
        self.working_dir = str(working_dir)
        self._temp = temp
        self._suffix = suffix or ""
        self._prefix = prefix or ""
        self._tmpdir = None
        self.path = None

    def __enter__(self):
        os.makedirs(self.working_dir, exist_ok=True)
        if self._temp:
            self._tmpdir = tempfile.TemporaryDirectory(suffix=self._suffix, prefix=self._prefix,
                                                       dir=self.working_dir)
            self.path = self._tmpdir.name
        else:
            self.path = os.path.join(self.working_dir, self._prefix + self._suffix)
            os.makedirs(self.path, exist_ok=True)
        return self.path

    def __exit__(self, exc_type, exc_value, traceback):
        if self._tmpdir is not None:
            self._tmpdir.cleanup()
            self._tmpdir = None
        return False


def remove(path):  # pragma: no cover - convenience
    shutil.rmtree(path, ignore_errors=True)
