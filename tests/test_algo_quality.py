"""Algorithm quality on the device sweep path: at an equal compute budget (the same number of
population steps), ASHA's best validation loss is no worse than random search's -- the reason
to run ASHA at all (reference: tests/functional/algos/test_algos.py:34-116 pins algorithm
quality on a noisy quadratic; this pins it on the MLP sweep the headline bench runs, with the
same trials-per-budget accounting as bench.py's best-loss@budget)."""
import pytest
import torch

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.models.mlp import MLPSweepTask
from metaopt_amd.ops.population import PopulationMLP
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import PopulationSweep

PRIORS = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(32, 128, discrete=True)",
          "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(16, 256, 4)"}
SYNC, INTERVALS, SLOTS = 16, 16, 8


def _best_at_budget(algorithms, seed, priors=PRIORS):
    torch.manual_seed(seed)
    data = TeacherClassification(n_train=2048, n_val=512, batch_size=128, seed=100 + seed)
    exp = build_experiment(f"quality-{list(algorithms)[0]}-{seed}", priors=priors,
                           algorithms=algorithms, storage=DocumentStorage(EphemeralDB()))
    pop = PopulationMLP(SLOTS, max_width=128, eval_batch=512, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=priors, max_width=128), data,
                            experiment=exp, sync_every=SYNC, ckpt_capacity=64)
    sweep.run(INTERVALS * SYNC)
    sweep.close()
    return sweep.best_within(INTERVALS * SYNC)


@pytest.mark.parametrize("seed", [0, 1])
def test_asha_no_worse_than_random_at_equal_budget(seed):
    asha, n_asha = _best_at_budget({"asha": {"seed": seed, "repetitions": float("inf")}}, seed)
    rand, n_rand = _best_at_budget({"random": {"seed": seed}}, seed)
    # random trains every trial at the top fidelity (256 steps = the whole budget); ASHA spends
    # the same population steps on many more, mostly short, rung evaluations
    assert n_asha > n_rand >= 1
    assert asha <= rand, (asha, rand)


SHORT = dict(PRIORS, **{"/steps": "fidelity(16, 64, 4)"})


@pytest.mark.parametrize("seed", [0, 2])
def test_async_asha_beats_random_when_random_finishes_many_trials(seed):
    """The regime where random search is not starved: the top fidelity (64 steps)
    is a quarter of the budget, so random search finishes >= 32 full-fidelity trials -- and
    asynchronous ASHA (promotion from the rung's running top 1/eta) still reaches the lower best
    loss at the same population steps.  (Measured over seeds 0-3: async ASHA 2.133 / 2.136 /
    2.120 / 2.191 vs random 2.209 / 2.170 / 2.199 / 2.205; the bounded reference brackets win 2
    of 4 -- profiles/round4.md.)"""
    asha, n_asha = _best_at_budget({"asha": {"seed": seed, "repetitions": float("inf"),
                                             "unbounded": True}}, seed, SHORT)
    rand, n_rand = _best_at_budget({"random": {"seed": seed}}, seed, SHORT)
    assert n_rand >= 32
    assert n_asha > n_rand
    assert asha <= rand, (asha, rand)
