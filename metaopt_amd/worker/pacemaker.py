"""Heartbeat thread for a running trial (reference: ``src/orion/core/worker/trial_pacemaker.py:14-52``).

Every ``wait_time`` seconds it refreshes the trial's ``heartbeat`` in storage; it stops on its own
once the trial is completed, interrupted or suspended, or when the heartbeat update fails (the
trial was taken over after being declared lost).
"""
from __future__ import annotations

import threading

STOPPED_STATUS = {"completed", "interrupted", "suspended", "broken"}


class TrialPacemaker(threading.Thread):
    def __init__(self, trial, wait_time=60, storage=None):
        super().__init__(daemon=True)
        from ..storage.protocol import get_storage
        self.stopped = threading.Event()
        self.trial = trial
        self.wait_time = wait_time
        self.storage = storage if storage is not None else get_storage()

    def stop(self):
        self.stopped.set()
        if self.is_alive():
            self.join()

    def run(self):
        while not self.stopped.wait(self.wait_time):
            self._monitor_trial()

    def _monitor_trial(self):
        trial = self.storage.get_trial(self.trial)
        if trial is None or trial.status in STOPPED_STATUS:
            self.stopped.set()
        elif not self.storage.update_heartbeat(trial):
            self.stopped.set()
