"""PopulationMLP on the PyTorch reference backend (CPU) and the population sweep engine."""
import numpy as np
import pytest
import torch

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.models.mlp import MLPSweepTask
from metaopt_amd.ops import reference as ref
from metaopt_amd.ops.population import MemberConfig, PopulationMLP, _ranges
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import PopulationSweep


@pytest.fixture(scope="module")
def data():
    return TeacherClassification(n_train=1024, n_val=256, batch_size=128, seed=7)


def test_rng_matches_python_int_hash():
    key = ref.rng_key(1234, 2, 17)
    idx = torch.arange(0, 1000, dtype=torch.int64)
    u = ref.rng_uniform(key, idx)
    for i in (0, 1, 500, 999):
        h = ref.fmix32(key ^ ((i * 0x9E3779B9) & ref.M32))
        assert float(u[i]) == (h >> 8) / 16777216.0
    assert 0.0 <= float(u.min()) and float(u.max()) < 1.0


def test_ranges():
    assert _ranges(np.array([2, 0, 3])).tolist() == [0, 1, 0, 1, 2]


def test_learns_and_isolates_members(data):
    pop = PopulationMLP(3, max_width=128, eval_batch=256, device="cpu")
    pop.set_member(0, MemberConfig(width=64, lr=0.1, seed=1))
    pop.set_member(2, MemberConfig(width=100, lr=0.0, seed=2))   # lr 0: must not move
    w_before = pop.layer_views(2)[0][0].clone()
    losses = []
    for step in range(30):
        pop.train_step(*data.batch(step))
        losses.append(pop.train_loss())
    losses = np.array(losses)
    assert losses[-5:, 0].mean() < losses[:5, 0].mean()
    assert torch.equal(pop.layer_views(2)[0][0], w_before)
    assert np.isnan(losses[:, 1]).all()


def test_padding_zero_and_init_deterministic():
    a = PopulationMLP(2, max_width=128, device="cpu")
    b = PopulationMLP(2, max_width=128, device="cpu")
    a.set_member(0, MemberConfig(width=70, lr=0.1, seed=9))
    b.set_member(1, MemberConfig(width=70, lr=0.1, seed=9))
    for (wa, ba), (wb, bb) in zip(a.layer_views(0), b.layer_views(1)):
        assert torch.equal(wa, wb) and torch.equal(ba, bb)
    w0, _ = a.layer_views(0)[0]
    assert float(w0[70:].abs().max()) == 0.0 and float(w0[:70, :784].abs().max()) > 0
    bound = 1 / np.sqrt(784)
    assert float(w0.abs().max()) <= bound + 1e-6


def test_checkpoint_roundtrip_and_copy(data):
    pop = PopulationMLP(3, max_width=128, eval_batch=256, device="cpu")
    pop.set_member(0, MemberConfig(width=64, lr=0.05, seed=3))
    for step in range(3):
        pop.train_step(*data.batch(step))
    st = pop.slot_state(0)
    assert st["t"] == 3 and st["p32"].numel() == pop.used_params(0)
    pop.load_slot_state(1, st)
    l1, _ = pop.evaluate(*data.validation())
    assert l1[0] == pytest.approx(l1[1], rel=1e-6)
    pop.copy_member(0, 2, lr=0.5)
    assert pop.members[2].lr == 0.5 and pop.steps_done(2) == 3
    sub, _ = pop.evaluate(*data.validation(), slots=[2])
    assert np.isnan(sub[0]) and not np.isnan(sub[2])


def test_adamw_reference_matches_torch_optim():
    torch.manual_seed(0)
    w = torch.randn(5, 3)
    g = torch.randn(5, 3)
    p = torch.nn.Parameter(w.clone())
    opt = torch.optim.AdamW([p], lr=0.01, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.1)
    m, v, w2 = torch.zeros_like(w), torch.zeros_like(w), w.clone()
    for t in range(1, 4):
        p.grad = g.clone()
        opt.step()
        ref.adamw_update(w2, m, v, g, 0.01, 0.9, 0.99, 1e-8, 0.1, t)
    assert torch.allclose(p.detach(), w2, atol=1e-6)


@pytest.mark.parametrize("pipelined", [None, False])
def test_sweep_asha_end_to_end(data, pipelined):
    """ASHA decides one interval behind the GPU by default (pipelined) and synchronously on
    request; both complete every trial and resume every promotion from its checkpoint."""
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(64, 128, discrete=True)",
              "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(16, 64, 2)"}
    storage = DocumentStorage(EphemeralDB())
    exp = build_experiment("sweep-test", priors=priors,
                           algorithms={"asha": {"seed": 1, "repetitions": float("inf")}},
                           max_trials=24, storage=storage)
    pop = PopulationMLP(6, max_width=128, eval_batch=256, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=priors, max_width=128), data,
                            experiment=exp, sync_every=16, pipelined=pipelined)
    assert sweep.pipelined == (pipelined is None)
    summary = sweep.run(1000)
    sweep.close()
    assert summary["completed"] == 24
    trials = exp.fetch_trials()
    assert len(trials) == 24 and all(t.status == "completed" for t in trials)
    budgets = sorted(t.params_dict["/steps"] for t in trials)
    assert budgets[0] == 16 and budgets[-1] >= 32  # promotions happened
    # every promotion continued from the lower-rung device checkpoint (none retrained)
    assert sweep.n_resumed == sum(1 for b in budgets if b > 16)
    assert sweep.n_resume_missing == 0
    assert exp.stats["best_evaluation"] == pytest.approx(summary["best_val_loss"])
    # the sweep writes trial documents directly: their ids are the Trial schema's md5 ids
    from metaopt_amd.core.trial import Trial
    docs = storage.database.read("trials", {})
    assert docs and all(Trial(**dict(d)).id == d["_id"] for d in docs)
    promoted = [d for d in docs if d["parents"]]
    assert all(p in {d["_id"] for d in docs} for t in promoted for p in t["parents"])


def test_sweep_marks_diverged_members_broken(data):
    priors = {"/lr": "loguniform(1e4, 1e5)", "/steps": "fidelity(16, 16, 2)"}
    storage = DocumentStorage(EphemeralDB())
    exp = build_experiment("sweep-nan", priors=priors, algorithms={"random": {"seed": 0}},
                           max_trials=4, storage=storage)
    pop = PopulationMLP(2, max_width=64, eval_batch=256, device="cpu")
    task = MLPSweepTask(priors=priors, width=64, max_width=64)
    sweep = PopulationSweep(pop, task, data, experiment=exp, sync_every=16)
    summary = sweep.run(200)
    sweep.close()
    statuses = [t.status for t in exp.fetch_trials()]
    assert summary["broken"] + summary["completed"] == 4
    assert statuses.count("broken") == summary["broken"]


def test_sweep_pbt_generations_resume_state(data):
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "choices([64])",
              "/steps": "fidelity(16, 48, 2)"}
    exp = build_experiment("sweep-pbt", priors=priors,
                           algorithms={"pbt": {"seed": 3, "population_size": 6, "interval": 16,
                                               "min_forking_population": 6,
                                               "freeze": ["/width"]}},
                           storage=DocumentStorage(EphemeralDB()))
    pop = PopulationMLP(6, max_width=64, eval_batch=256, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=priors, max_width=64), data,
                            experiment=exp, sync_every=16)
    assert not sweep.pipelined              # PBT generations decide synchronously
    summary = sweep.run(200)
    sweep.close()
    assert sweep.done and summary["completed"] == 18
    assert sweep.global_step == 48          # 3 generations x 16 steps, no retraining
    assert sweep.n_resumed == 12 and sweep.n_resume_missing == 0
    trials = exp.fetch_trials()
    ids = {t.id for t in trials}
    children = [t for t in trials if t.parents]
    assert len(children) == 12 and all(t.parents[0] in ids for t in children)


def test_sweep_point_key_matches_task_key(data):
    """The sweep derives configuration keys from points with a format template; they must be
    the task's ``param_key`` exactly (promotion lookup and per-configuration init seeds)."""
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(64, 128, discrete=True)",
              "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(16, 64, 2)"}
    exp = build_experiment("key-test", priors=priors, algorithms={"random": {"seed": 2}},
                           max_trials=4, storage=DocumentStorage(EphemeralDB()))
    task = MLPSweepTask(priors=priors, max_width=128)
    sweep = PopulationSweep(PopulationMLP(2, max_width=128, device="cpu"), task, data,
                            experiment=exp, sync_every=16)
    assert sweep._pkey_tmpl is not None
    for point in exp.algorithms.suggest(8):
        params = dict(zip(sweep._dim_names, point))
        assert sweep._point_key(point) == task.key(params)
    sweep.close()


def test_bf16_momentum_reference_update():
    """The bf16 momentum buffer: one RNE rounding of the f32 update, which then drives W."""
    import torch
    from metaopt_amd.ops import reference as ref
    w = torch.tensor([1.0, -2.0, 0.5])
    g = torch.tensor([0.3, 0.1, -0.7])
    m16 = torch.tensor([0.2, -0.4, 1.0]).to(torch.bfloat16)
    m_exact = m16.float() * 0.9 + (g + 1e-3 * w)
    w_exp = w - 0.1 * m_exact.to(torch.bfloat16).float()
    ref.sgd_update(w, m16, g, 0.1, 0.9, 1e-3)
    assert m16.dtype == torch.bfloat16
    assert torch.equal(m16, m_exact.to(torch.bfloat16))
    assert torch.allclose(w, w_exp, rtol=0, atol=1e-7)


def test_bf16_momentum_population_trains_on_cpu():
    import numpy as np
    from metaopt_amd.models.data import TeacherClassification
    from metaopt_amd.ops.population import MemberConfig, PopulationMLP
    data = TeacherClassification(n_train=1024, n_val=128, batch_size=128, seed=0)
    pop = PopulationMLP(2, max_width=64, eval_batch=128, device="cpu", momentum_dtype="bf16")
    assert pop.m32.dtype == __import__("torch").bfloat16
    pop.set_member(0, MemberConfig(width=64, lr=0.1, seed=1))
    losses = []
    for step in range(8):
        pop.train_step(*data.batch(step))
        losses.append(pop.train_loss()[0])
    assert np.isfinite(losses).all() and losses[-1] < losses[0]
    st = pop.slot_state(0)
    assert st["m32"].dtype == __import__("torch").bfloat16


def test_work_tables_are_bounds_checked():
    """Every table a launch reads is validated against the buffers before use; a corrupted
    descriptor is refused on the host instead of reaching a kernel."""
    import numpy as np
    import pytest
    from metaopt_amd.ops.population import MemberConfig, PopulationMLP
    pop = PopulationMLP(3, max_width=128, eval_batch=128, device="cpu")
    pop.set_member(1, MemberConfig(width=100, lr=0.1, seed=1))
    tb = pop._build_tables(128)
    tl = tb["tl_np"].copy()
    tl["w_off"][1 * pop.L + 1] = pop.capacity * pop.slot_params        # past the end
    with pytest.raises(ValueError, match="weights outside"):
        pop._validate_tables(tl, tb["fwd_np"], tb["bwd_np"], 128)
    fwd = [w.copy() for w in tb["fwd_np"]]
    fwd[0][0, 1] = 99                                                   # tile index too large
    with pytest.raises(ValueError, match="tile out of range"):
        pop._validate_tables(tb["tl_np"], fwd, tb["bwd_np"], 128)
    fwd = [w.copy() for w in tb["fwd_np"]]
    fwd[1][0, 0] = 0                                                    # an empty slot's layer
    with pytest.raises(ValueError, match="missing trial-layer"):
        pop._validate_tables(tb["tl_np"], fwd, tb["bwd_np"], 128)


def test_init_descriptors_match_the_layer_layout():
    """The vectorised member-initialisation descriptors equal the per-layer layout
    (layer_dims / real_dims / param_offsets) row for row, logistic regression included."""
    import numpy as np
    from metaopt_amd.ops.population import MemberConfig, PopulationMLP
    for n_hidden, widths in ((3, (64, 100, 1, 257)), (0, (64,))):
        pop = PopulationMLP(6, in_features=784 if n_hidden else 2,
                            num_classes=10 if n_hidden else 2, n_hidden=n_hidden,
                            max_width=320, device="cpu")
        slots = [1, 3, 4, 5][:len(widths)]
        for s, w in zip(slots, widths):
            pop.set_member(s, MemberConfig(width=w, lr=0.1, seed=1000 + s), init=False)
        got = pop._init_descs(slots)
        rows = []
        for s in slots:
            cfg = pop.members[s]
            base = pop.slot_base(s)
            for l, ((k, n), (kr, nr), (wo, bo)) in enumerate(zip(
                    pop.layer_dims(cfg.width), pop.real_dims(cfg.width),
                    pop.param_offsets(cfg.width))):
                rows.append((base + wo, base + bo, k, n, kr, nr, cfg.seed, l,
                             np.float32(1.0) / np.sqrt(np.float32(kr)), 0))
        want = np.array(rows, dtype=got.dtype)
        assert (got == want).all()


def test_per_member_batch_size_trains_on_its_own_rows():
    """A member with ``batch_size`` 128 inside a 256-row population follows exactly the member
    of a 128-row population fed the first 128 rows (reference backend); the loss statistics are
    means over each member's own rows, also for a snapshot taken before its slot was reused."""
    data = TeacherClassification(n_train=2048, n_val=256, batch_size=256, seed=8)
    big = PopulationMLP(3, max_width=128, batch_size=256, device="cpu")
    small = PopulationMLP(1, max_width=128, batch_size=128, device="cpu")
    cfg = MemberConfig(width=96, lr=0.1, seed=4, dropout=0.2)
    big.set_member(0, MemberConfig(**dict(cfg.to_dict(), batch_size=128)))
    big.set_member(2, MemberConfig(width=64, lr=0.1, seed=5))          # 0: the population's 256
    small.set_member(0, cfg)
    for step in range(4):
        x, y = data.batch(step)
        big.train_step(x, y)
        small.train_step(x[:128], y[:128])
    assert big.train_loss()[0] == pytest.approx(small.train_loss()[0], rel=1e-6)
    for (wa, ba), (wb, bb) in zip(big.layer_views(0), small.layer_views(0)):
        assert torch.allclose(wa, wb, atol=1e-7) and torch.allclose(ba, bb, atol=1e-7)
    # snapshot rows survive a slot reuse with another batch size
    snap = big.stats_snapshot_async()
    raw = snap.get().copy()
    big.remove_member(0)
    big.set_member(0, MemberConfig(width=64, lr=0.1, seed=6, batch_size=256))
    big._refresh()
    then, _, _ = big.raw_results(raw, None, snap.rows)
    now, _, _ = big.raw_results(raw, None)
    assert then[0] == pytest.approx(2 * now[0])


def test_member_batch_size_is_validated():
    pop = PopulationMLP(2, max_width=128, batch_size=256, device="cpu")
    for bad in (64, 200, 384):
        with pytest.raises(ValueError, match="batch_size"):
            pop.set_member(0, MemberConfig(width=64, lr=0.1, batch_size=bad))
    pop.set_member(0, MemberConfig(width=64, lr=0.1, batch_size=128))
    with pytest.raises(ValueError, match="batch_size"):
        pop.update_hparams(0, batch_size=512)
    pop.update_hparams(0, batch_size=256)
    tb = pop._build_tables(256, member_rows=True)
    assert (tb["tl_np"]["rows"][:pop.L] == 256).all()
    with pytest.raises(ValueError, match="multiples of 128"):
        PopulationMLP(2, batch_size=100, device="cpu")
    tl = tb["tl_np"].copy()
    tl["rows"][0] = 384                                 # more rows than the launch holds
    with pytest.raises(ValueError, match="trial rows"):
        pop._validate_tables(tl, tb["fwd_np"], tb["bwd_np"], 256)


def test_sweep_tunes_the_batch_size():
    """``/batch_size`` as a searched hyper-parameter: the mlp task sizes the population for the
    largest choice, each trial trains on its own rows, promotions keep the batch size."""
    from metaopt_amd.worker import tasks
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(64, 128, discrete=True)",
              "/batch_size": "choices([128, 256])", "/steps": "fidelity(16, 32, 2)"}
    task, pop, data = tasks.get("mlp").build(4, "cpu", 0, priors=priors, state_dtype="fp32")
    assert pop.batch_size == 256 and data.batch_size == 256
    storage = DocumentStorage(EphemeralDB())
    exp = build_experiment("sweep-batch", priors=priors,
                           algorithms={"asha": {"seed": 2, "repetitions": float("inf")}},
                           max_trials=10, storage=storage)
    seen = set()
    real = pop.set_member

    def spy(slot, cfg, init=True):
        seen.add(pop.member_rows(cfg))
        return real(slot, cfg, init)
    pop.set_member = spy
    sweep = PopulationSweep(pop, task, data, experiment=exp, sync_every=16)
    summary = sweep.run(1000)
    sweep.close()
    assert summary["completed"] == 10
    assert seen == {128, 256}
    for bad in ("choices([100, 256])", "uniform(128, 256)"):
        with pytest.raises(ValueError, match="batch_size"):
            tasks._max_batch({"/batch_size": bad})
