"""Population ResNet on the CPU reference backend and a TPE sweep over it (config 3, toy size)."""
import numpy as np
import torch

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.resnet import PopulationResNet, ResNetSweepTask, SyntheticCIFAR
from metaopt_amd.ops import conv as cops
from metaopt_amd.ops.population import MemberConfig
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import PopulationSweep


def _pop(P=2):
    return PopulationResNet(P, batch_size=16, device="cpu", blocks_per_stage=1, image_size=16)


def _data():
    return SyntheticCIFAR(n_train=16 * 8, n_val=32, batch_size=16, image_size=16)


def test_im2col_reference_is_a_convolution():
    torch.manual_seed(0)
    x = torch.randn(2, 9, 9, 8)
    w = torch.randn(1, 72, 16)
    for stride in (1, 2):
        out = cops.conv3x3_ref(x, w, 1, stride)
        wt = w[0].view(3, 3, 8, 16).permute(3, 2, 0, 1)          # [Cout, Cin, kh, kw]
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), wt, stride=stride, padding=1)
        torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, rtol=1e-4, atol=1e-4)


def test_resnet_learns_isolated_members_and_running_stats():
    pop = _pop()
    pop.set_member(0, MemberConfig(width=0, lr=0.05, momentum=0.9, seed=1))
    pop.set_member(1, MemberConfig(width=0, lr=0.0, momentum=0.9, seed=2))
    frozen = pop.W["s2b0c2.w"][1].detach().clone()
    data = _data()
    before = pop.A["conv0.running"][0].clone()
    for s in range(6):
        pop.train_step(*data.batch(s))
    assert torch.equal(frozen, pop.W["s2b0c2.w"][1].detach())
    assert not torch.equal(before, pop.A["conv0.running"][0])   # running stats move in train
    vl, acc = pop.evaluate(*data.validation())
    assert np.isfinite(vl).all() and ((acc >= 0) & (acc <= 1)).all()


def test_resnet_checkpoint_includes_running_stats():
    pop = _pop()
    for s in range(2):
        pop.set_member(s, MemberConfig(width=0, lr=0.05, seed=s))
    data = _data()
    pop.train_step(*data.batch(0))
    pop.alloc_ckpt_pool(2)
    meta = pop.save_states([(0, 0)])[0]
    ref = pop.slot_state(0)
    pop.train_step(*data.batch(1))
    pop.load_states([(1, meta)])
    got = pop.slot_state(1)
    for k in ("p32", "m32", "aux"):
        assert torch.equal(got[k], ref[k]), k
    st = pop.unpack_state(pop.pack_state(pop.pool_state(meta)))
    assert torch.equal(st["aux"], ref["aux"]) and st["t"] == 1


def test_tpe_sweep_over_resnet_members():
    priors = {"/lr": "loguniform(0.01, 0.3)", "/momentum": "uniform(0.5, 0.95)"}
    exp = build_experiment("resnet-tpe", priors=priors,
                           algorithms={"tpe": {"seed": 1, "n_initial_points": 4}},
                           max_trials=6, storage=DocumentStorage(EphemeralDB()))
    pop = _pop(3)
    task = ResNetSweepTask(priors=priors, steps=4)
    sweep = PopulationSweep(pop, task, _data(), experiment=exp, sync_every=4, ckpt_capacity=4)
    summary = sweep.run(40)
    sweep.close()
    assert summary["completed"] == 6 and sweep.done
    trials = exp.fetch_trials()
    assert all(t.status == "completed" and any(r.name == "val_acc" for r in t.results)
               for t in trials)
