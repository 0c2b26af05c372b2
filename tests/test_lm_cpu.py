"""Population LM on the CPU reference backend: learning, member isolation, checkpoints, and a
PBT sweep over LM members (BASELINE.json config 5 at toy scale)."""
import numpy as np
import torch

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.llama import LMSweepTask, PopulationLM, SyntheticLM
from metaopt_amd.ops.population import MemberConfig
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import PopulationSweep


def _data():
    return SyntheticLM(512, 64, 4, n_tokens=1 << 14, seed=0)


def test_lm_learns_and_isolates():
    pop = PopulationLM(2, "micro", batch_size=4, device="cpu")
    pop.set_member(0, MemberConfig(width=128, lr=3e-3, seed=1, beta2=0.95))
    pop.set_member(1, MemberConfig(width=128, lr=0.0, seed=2, beta2=0.95))
    frozen = pop.W["l1.wdown"][1].detach().clone()
    data = _data()
    first = None
    for s in range(20):
        pop.train_step(*data.batch(s))
        first = pop.train_loss() if first is None else first
    last = pop.train_loss()
    assert last[0] < first[0] - 0.5
    assert torch.equal(frozen, pop.W["l1.wdown"][1].detach())
    vl, ppl = pop.evaluate(*data.validation())
    assert np.isfinite(vl).all() and np.allclose(ppl, np.exp(vl))


def test_lm_checkpoint_pool_roundtrip():
    pop = PopulationLM(2, "micro", batch_size=4, device="cpu")
    pop.set_member(0, MemberConfig(width=128, lr=3e-3, seed=1, beta2=0.95))
    pop.set_member(1, MemberConfig(width=128, lr=1e-3, seed=2, beta2=0.95))
    data = _data()
    pop.train_step(*data.batch(0))
    pop.alloc_ckpt_pool(2)
    meta = pop.save_states([(0, 1)])[0]
    ref = pop.slot_state(0)
    pop.train_step(*data.batch(1))
    pop.load_states([(1, meta)])
    got = pop.slot_state(1)
    assert got["t"] == ref["t"] == 1
    for k in ("p32", "m32", "v32"):
        assert torch.equal(got[k], ref[k])
    packed = pop.pack_state(pop.pool_state(meta))
    st = pop.unpack_state(packed)
    assert st["t"] == 1 and torch.equal(st["p32"], ref["p32"])


def test_pbt_sweep_over_lm_members():
    priors = {"/lr": "loguniform(1e-4, 3e-3)", "/weight_decay": "loguniform(1e-3, 0.1)",
              "/steps": "fidelity(8, 24, 2)"}
    exp = build_experiment("lm-pbt", priors=priors,
                           algorithms={"pbt": {"seed": 1, "population_size": 4, "interval": 8,
                                               "min_forking_population": 4}},
                           storage=DocumentStorage(EphemeralDB()))
    pop = PopulationLM(4, "micro", batch_size=2, device="cpu")
    task = LMSweepTask(priors=priors, d_model=128)
    data = SyntheticLM(512, 64, 2, n_tokens=1 << 13, seed=0)
    sweep = PopulationSweep(pop, task, data, experiment=exp, sync_every=8, ckpt_capacity=8)
    summary = sweep.run(100)
    sweep.close()
    assert sweep.done and summary["completed"] == 12
    assert sweep.global_step == 24 and sweep.n_resumed == 8 and sweep.n_resume_missing == 0
    trials = exp.fetch_trials()
    assert all(t.status == "completed" for t in trials)
    assert all(any(r.name == "val_ppl" for r in t.results) for t in trials)
