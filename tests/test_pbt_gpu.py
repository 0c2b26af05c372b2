"""Config 5 on the device: a PBT sweep over LM members (the 2-layer ``tiny-2layer`` preset, the
same code path as the 125M bench) through at least two exploit rounds.

Checked at every checkpoint load of the sweep (exploit copies included), right after the copy:
the destination slot's bf16 working weights, the low half of the split f32 master, both AdamW
moments, the auxiliary state and the step counter equal, bit for bit, the source slot's state
at the moment it was checkpointed.  Then: training stays finite, every trial of generation > 0
names its parent trial (``parents``, reference ``src/orion/core/worker/trial.py:159-160``), and
the exploited children carry perturbed (explored) hyper-parameters.
"""
import math

import pytest
import torch



def _raw(pop, slot):
    """Every state buffer of one slot, as raw bits (bf16 / int16 -> int16, f32 -> int32)."""
    sl = pop._slices(slot)
    cat = lambda b: torch.cat([b[x] for x in sl]).clone()   # noqa: E731
    bits = lambda t: t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)  # noqa
    out = {"p16": bits(cat(pop.p16)), "master": bits(cat(pop.master_buf)), "m": bits(cat(pop.m)),
           "aux": bits(pop._aux_of(slot).clone()), "t": int(pop.hp[slot]["t"])}
    if pop.v.numel():
        out["v"] = bits(cat(pop.v))
    return out


def _pbt_sweep(dev, preset, seq_len):
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.llama import LMSweepTask, PopulationLM, SyntheticLM
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import PopulationSweep

    P, interval = 6, 8
    priors = {"/lr": "loguniform(1e-4, 3e-3)", "/weight_decay": "loguniform(1e-3, 0.1)",
              "/beta1": "uniform(0.8, 0.95)", "/steps": f"fidelity({interval}, {3 * interval}, 2)"}
    exp = build_experiment("pbt-gpu", priors=priors,
                           algorithms={"pbt": {"seed": 3, "population_size": P,
                                               "interval": interval,
                                               "min_forking_population": P,
                                               # bottom third exploits: 2 per generation
                                               "truncation_quantile": 0.66,
                                               "candidate_pool_ratio": 0.34}},
                           storage=DocumentStorage(EphemeralDB()))
    pop = PopulationLM(P, preset, batch_size=4, seq_len=seq_len, device=dev,
                       moment_dtype=torch.bfloat16 if dev == "cuda" else None)
    task = LMSweepTask(priors=priors, d_model=pop.cfg.d_model)
    data = SyntheticLM(pop.cfg.vocab, seq_len, 4, n_tokens=1 << 16, seed=0, device=dev)
    sweep = PopulationSweep(pop, task, data, experiment=exp, sync_every=interval,
                            ckpt_capacity=2 * P)

    saved, checked = {}, []
    orig_save, orig_load = pop.save_states, pop.load_states

    sync = torch.cuda.synchronize if dev == "cuda" else (lambda: None)

    def save(pairs):
        sync()
        for s, idx in pairs:
            saved[idx] = _raw(pop, s)
        return orig_save(pairs)

    def load(pairs):
        orig_load(pairs)
        sync()
        for s, meta in pairs:
            got, ref = _raw(pop, s), saved[meta["ck"]]
            assert got["t"] == ref["t"] > 0
            for k in ref:
                if k != "t":
                    assert torch.equal(got[k], ref[k]), (k, s, meta["ck"])
            checked.append((s, meta["ck"]))

    pop.save_states, pop.load_states = save, load
    summary = sweep.run(10 * interval)
    sweep.close()

    algo = sweep.algorithm.algorithm
    assert sweep.done and summary["completed"] == 3 * P
    assert sweep.n_resume_missing == 0
    assert len(checked) == sweep.n_resumed == 2 * P          # every successor resumed a copy
    assert len(algo.exploit_log) >= 2                          # >= 2 exploits ...
    assert len({g for g, _, _ in algo.exploit_log}) == 2       # ... in both exploit rounds
    trials = exp.fetch_trials()
    assert len(trials) == 3 * P and all(t.status == "completed" for t in trials)
    assert all(math.isfinite(t.objective.value) for t in trials)
    by_id = {t.id: t for t in trials}
    steps = lambda t: t.params_dict["/steps"]                                   # noqa: E731
    hp = lambda t: {k: v for k, v in t.params_dict.items() if k != "/steps"}    # noqa: E731
    children = [t for t in trials if steps(t) > interval]
    assert len(children) == 2 * P
    explored = 0
    for t in children:
        assert len(t.parents) == 1 and t.parents[0] in by_id
        parent = by_id[t.parents[0]]
        assert steps(parent) == steps(t) - interval
        explored += hp(parent) != hp(t)
    assert explored == sum(n for _, n in algo.exploit_counts().values()) >= 2
    return pop


@pytest.mark.gpu
def test_pbt_sweep_exploit_copies_are_bitwise_and_lineage_is_recorded():
    """On the GPU: HIP kernels, split f32 master (bf16 high half + int16 low half), bf16 first
    moment widened into the f32 checkpoint pool and narrowed back."""
    pop = _pbt_sweep("cuda", "tiny-2layer", 128)
    assert pop.backend == "hip" and pop.split and pop.m.dtype == torch.bfloat16


def test_pbt_sweep_exploit_copies_cpu_reference():
    pop = _pbt_sweep("cpu", "micro", 64)
    assert pop.backend == "torch"
