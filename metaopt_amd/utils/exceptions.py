"""Framework exceptions (reference: ``src/orion/core/utils/exceptions.py:12-27``)."""


class NoConfigurationError(Exception):
    """An experiment is asked for by name but has no configuration (and none was given)."""


class CheckError(Exception):
    """A ``db test`` check stage failed."""


class RaceCondition(Exception):
    """Two workers raced to create/branch the same experiment version."""


class BrokenExperiment(RuntimeError):
    """Too many broken trials (``worker.max_broken``)."""


class SampleTimeout(RuntimeError):
    """The algorithm could not produce new trials within ``worker.max_idle_time``."""


class WaitingForTrials(RuntimeError):
    """Nothing is reservable yet, but other workers still have trials in flight."""
