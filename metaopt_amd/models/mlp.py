"""The 4-layer MLP sweep task (BASELINE.json configs 1 and 2).

Maps a trial's parameters to a :class:`~metaopt_amd.ops.population.MemberConfig` of the device
population, and names the search space the benchmark sweeps:

* ``/lr ~ loguniform(1e-3, 1.0)`` -- SGD learning rate (momentum 0.9, weight decay 5e-4 fixed);
* ``/width ~ loguniform(64, 1024, discrete=True)`` -- hidden width of the 3 ReLU layers;
* ``/dropout ~ uniform(0, 0.5)`` -- dropout after each hidden layer;
* ``/steps ~ fidelity(32, 2048, 4)`` -- training budget in optimizer steps (ASHA rungs 32, 128, 512,
  2048);
* optional ``/batch_size`` (e.g. ``choices([128, 256, 512])``) -- rows per step of the trial, a
  multiple of 128; the population is sized for the largest value the prior can take and a trial
  trains on the first rows of each minibatch (``MemberConfig.batch_size``).

Config 1 (logistic regression, CPU) is the same task with ``n_hidden=0`` and a 2-HP space
(``/lr``, ``/weight_decay``).
"""
from __future__ import annotations

import hashlib

import numpy as np
from dataclasses import dataclass, field
from typing import ClassVar, Dict, Optional

from ..ops.population import MemberConfig

MLP_PRIORS = {
    "/lr": "loguniform(1e-3, 1.0)",
    "/width": "loguniform(64, 1024, discrete=True)",
    "/dropout": "uniform(0, 0.5)",
    "/steps": "fidelity(32, 2048, 4)",
}

LOGREG_PRIORS = {
    "/lr": "loguniform(1e-3, 1.0)",
    "/weight_decay": "loguniform(1e-6, 1e-1)",
    "/steps": "fidelity(64, 256, 2)",
}


def param_key(params: Dict, fidelity_name: str) -> str:
    """Identity of a configuration regardless of its budget (the ASHA promotion key)."""
    items = sorted((k, _plain(v)) for k, v in params.items() if k != fidelity_name)
    return hashlib.md5(repr(items).encode("utf-8")).hexdigest()


def _plain(v):
    """numpy scalars/arrays -> Python values, so equal configurations hash equally."""
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


@dataclass
class MLPSweepTask:
    priors: Dict[str, str] = field(default_factory=lambda: dict(MLP_PRIORS))
    # key(params) == param_key(params, fidelity): the sweep may derive it from points directly
    key_by_params: ClassVar[bool] = True
    fidelity: str = "/steps"
    momentum: float = 0.9
    weight_decay: float = 5e-4
    width: int = 256          # used when the space has no /width
    n_hidden: int = 3
    in_features: int = 784
    num_classes: int = 10
    max_width: int = 1024
    steps: int = 256          # budget of every trial when the space has no /steps fidelity

    def member_config(self, params: Dict, seed: int) -> MemberConfig:
        return MemberConfig(
            width=int(params.get("/width", self.width)),
            lr=float(params["/lr"]),
            momentum=float(params.get("/momentum", self.momentum)),
            weight_decay=float(params.get("/weight_decay", self.weight_decay)),
            dropout=float(params.get("/dropout", 0.0)) if self.n_hidden > 0 else 0.0,
            seed=int(seed) & 0x7FFFFFFF,
            batch_size=self.batch_rows(params),
        )

    def batch_rows(self, params: Dict) -> int:
        """Rows per step of the trial (0: the population's batch size)."""
        return int(params.get("/batch_size", 0))

    def member_row(self, params: Dict, seed: int) -> tuple:
        """(width, lr, momentum, weight decay, dropout, seed) of :meth:`member_config` without
        building the dataclass (the sweep places thousands of members per sync)."""
        g = params.get
        return (int(g("/width", self.width)), float(params["/lr"]),
                float(g("/momentum", self.momentum)),
                float(g("/weight_decay", self.weight_decay)),
                float(g("/dropout", 0.0)) if self.n_hidden > 0 else 0.0,
                int(seed) & 0x7FFFFFFF)

    def point_row_fn(self, names):
        """``(row, budget, batch)`` functions of a suggested point in ``names`` order: the
        :meth:`member_row`, :meth:`budget` and :meth:`batch_rows` of ``dict(zip(names, point))``
        without building the dict (rank 0 places up to thousands of trials per sync); None
        when a dimension outside this task's hyper-parameters is present."""
        known = {"/lr", "/width", "/momentum", "/weight_decay", "/dropout", "/batch_size",
                 self.fidelity}
        if "/lr" not in names or any(n not in known for n in names):
            return None
        ix = {n: i for i, n in enumerate(names)}
        i_lr = ix["/lr"]
        i_w, i_m = ix.get("/width"), ix.get("/momentum")
        i_wd, i_d = ix.get("/weight_decay"), ix.get("/dropout")
        i_f, i_b = ix.get(self.fidelity), ix.get("/batch_size")
        width, mom, wd, steps = self.width, self.momentum, self.weight_decay, self.steps
        hidden = self.n_hidden > 0

        def row(p, seed):
            return (int(p[i_w]) if i_w is not None else int(width), float(p[i_lr]),
                    float(p[i_m]) if i_m is not None else float(mom),
                    float(p[i_wd]) if i_wd is not None else float(wd),
                    float(p[i_d]) if (i_d is not None and hidden) else 0.0,
                    int(seed) & 0x7FFFFFFF)

        def budget(p):
            return int(p[i_f]) if i_f is not None else int(steps)

        def batch(p):
            return int(p[i_b]) if i_b is not None else 0

        return row, budget, batch

    def budget(self, params: Dict) -> int:
        return int(params.get(self.fidelity, self.steps))

    def key(self, params: Dict) -> str:
        return param_key(params, self.fidelity)

    @staticmethod
    def seed_of(key: str) -> int:
        """Deterministic per-configuration seed (same weights init when a trial is re-run)."""
        return int(key[:8], 16)
