"""Test harness shipped with the package (reference: ``src/orion/core/utils/tests.py:28-212``,
``OrionState``): a context manager that installs a fresh storage as the process-wide one, seeds
it with experiment / trial / lie documents, and restores the previous storage on exit -- so tests
of code that calls ``get_storage()`` run against a known, isolated database.

    with MoptState(experiments=[exp_cfg], trials=[trial_doc], storage="pickleddb") as st:
        ...   # st.storage is the installed DocumentStorage
"""
from __future__ import annotations

import copy
import datetime
import os
import tempfile
from typing import List, Optional

from ..storage import protocol
from ..storage.database import EphemeralDB, create_database
from ..storage.protocol import DocumentStorage


class MockDatetime(datetime.datetime):
    """``datetime.datetime`` whose ``utcnow()`` is frozen (deterministic documents)."""

    frozen = datetime.datetime(1903, 4, 25, 0, 0, 0)

    @classmethod
    def utcnow(cls):  # noqa: D102
        return cls.frozen


class MoptState:
    """Swap in a seeded storage for the duration of a ``with`` block."""

    def __init__(self, experiments: Optional[List[dict]] = None,
                 trials: Optional[List[dict]] = None, lies: Optional[List[dict]] = None,
                 storage: str = "ephemeraldb"):
        self.experiments = copy.deepcopy(experiments or [])
        self.trials = copy.deepcopy(trials or [])
        self.lies = copy.deepcopy(lies or [])
        self.kind = storage.lower()
        self.storage: Optional[DocumentStorage] = None
        self._saved = None
        self._tmp = None

    def _make_db(self):
        if self.kind == "ephemeraldb":
            return EphemeralDB()
        if self.kind == "pickleddb":
            fd, self._tmp = tempfile.mkstemp(suffix=".pkl", prefix="mopt_state_")
            os.close(fd)
            os.remove(self._tmp)
            return create_database("pickleddb", host=self._tmp)
        raise ValueError(f"unsupported test storage {self.kind!r}")

    def __enter__(self) -> "MoptState":
        self._saved = getattr(protocol, "_STORAGE", None)
        self.storage = DocumentStorage(self._make_db())
        protocol._STORAGE = self.storage
        db = self.storage.database
        for name, docs in (("experiments", self.experiments), ("trials", self.trials),
                           ("lying_trials", self.lies)):
            if docs:
                db.write(name, copy.deepcopy(docs))
        return self

    def __exit__(self, *exc):
        protocol._STORAGE = self._saved
        if self._tmp:
            for path in (self._tmp, self._tmp + ".lock"):
                if os.path.exists(path):
                    os.remove(path)
        return False
