"""Observed-trial bookkeeping (reference: ``src/orion/core/worker/trials_history.py:14-40``):
the set of observed ids and the current lineage "children" recorded as new trials' ``parents``."""
from __future__ import annotations


class TrialsHistory:
    def __init__(self):
        self.children = []
        self.ids = set()

    def __contains__(self, trial):
        return trial.id in self.ids

    def update(self, trials):
        descendants = set(self.children)
        for t in trials:
            descendants -= set(t.parents)
            descendants.add(t.id)
        self.ids |= descendants
        self.children = sorted(descendants)
