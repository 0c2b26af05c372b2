"""Staggered start of large populations (worker/population_sweep.py ``stagger``): the first fill
of an empty population is spread over several syncs so the members' budgets do not all end at
the same sync (rank 0's decision work per sync stays near the mean instead of a periodic burst).
Rank 0's decision is driven directly on simulated status blocks, as in scripts/profile_decide.py.
"""
import numpy as np
import torch

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.mlp import MLP_PRIORS, MLPSweepTask
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import NEW, PopulationSweep


class _Pop:
    def __init__(self, capacity):
        self.capacity = capacity
        self.device = torch.device("cpu")

    def alloc_ckpt_pool(self, n):
        pass


class _Comm:
    def __init__(self, world):
        self.world_size, self.rank, self.is_root, self.distributed = world, 0, True, False
        self.device = torch.device("cpu")

    def broadcast_object(self, obj, src=0):
        return obj

    def all_gather_object(self, obj):
        return [obj]


def _sweep(world, P, stagger=None):
    exp = build_experiment("stagger", priors=dict(MLP_PRIORS),
                           algorithms={"random": {"seed": 0}},
                           storage=DocumentStorage(EphemeralDB()), pool_size=P)
    return PopulationSweep(_Pop(P), MLPSweepTask(priors=dict(MLP_PRIORS), max_width=1024),
                           data=None, comm=_Comm(world), experiment=exp, sync_every=32,
                           pipelined=False, writer="inline", stagger=stagger)


def _busy_after_fills(sw, world, P, n):
    rows = world * P
    gathered = np.zeros((rows, 9))
    gathered[:, 0] = -1
    gathered[:, 4] = -1
    busy = []
    for _ in range(n):
        assign = sw._decide(gathered)
        new = np.flatnonzero(assign[:rows, 0] == NEW)
        gathered[new, 0] = assign[new, 1]
        gathered[new, 2] = assign[new, 8]          # budget; steps stay 0: nobody finishes
        busy.append(int((gathered[:, 0] >= 0).sum()))
    return busy


def test_large_population_fills_over_four_syncs_balanced_across_ranks():
    world, P = 8, 256
    sw = _sweep(world, P)
    assert sw.stagger == 4
    busy = _busy_after_fills(sw, world, P, 5)
    assert busy == [512, 1024, 1536, 2048, 2048]
    sw.close()


def test_small_population_fills_at_once():
    world, P = 2, 256
    sw = _sweep(world, P)
    assert sw.stagger == 1
    assert _busy_after_fills(sw, world, P, 2) == [512, 512]
    sw.close()


def test_first_cohort_spread_over_ranks():
    world, P = 8, 256
    sw = _sweep(world, P, stagger=4)
    rows = world * P
    gathered = np.zeros((rows, 9))
    gathered[:, 0] = -1
    gathered[:, 4] = -1
    assign = sw._decide(gathered)
    per_rank = (assign[:rows, 0] == NEW).reshape(world, P).sum(1)
    assert per_rank.tolist() == [64] * world       # every GPU busy from the first interval
    sw.close()
