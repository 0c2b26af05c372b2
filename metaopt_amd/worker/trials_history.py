"""Which trials the producer has already fed to the algorithm, and the current lineage frontier.

Semantics of the reference's ``TrialsHistory`` (``src/orion/core/worker/trials_history.py``):
``trial in history`` tells whether ``trial`` was observed; ``update(trials)`` observes a batch,
where each trial replaces its parents on the *frontier* (``children``: the ids new trials list as
their ``parents``).  Kept as a frontier set updated in place rather than rebuilt per call.
"""
from __future__ import annotations

from typing import Iterable, List, Set


class TrialsHistory:
    def __init__(self):
        self._seen: Set[str] = set()
        self._frontier: Set[str] = set()

    @property
    def ids(self) -> Set[str]:
        return self._seen

    @property
    def children(self) -> List[str]:
        """Sorted ids of the frontier (the lineage leaves after the last update)."""
        return sorted(self._frontier)

    def __contains__(self, trial) -> bool:
        return trial.id in self._seen

    def update(self, trials: Iterable) -> None:
        for trial in trials:
            self._frontier.difference_update(trial.parents)
            self._frontier.add(trial.id)
        self._seen.update(self._frontier)
