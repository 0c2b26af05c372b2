"""Named device-population tasks: what ``mopt sweep`` and ``scripts/bench_configs.py`` train.

Each entry builds, for one rank, the trial->member mapping (task), the device population and
the synthetic dataset of a BASELINE.json configuration:

=========  ===============================================================  =======================
name       model / data                                                      default algorithm
=========  ===============================================================  =======================
logreg     logistic regression, 2-D synthetic 2-class data (config 1)        random
mlp        4-layer MLP 784-w-w-w-10, MNIST-shaped teacher data (config 2)    asha
resnet20   ResNet-20, CIFAR-shaped teacher data (config 3)                   tpe
lm-125m    Llama-style 125M LM, synthetic bigram tokens (config 5)          pbt
lm-tiny    2-layer LM (d 256), same data (config 4's model)                  pbt
=========  ===============================================================  =======================
"""
from __future__ import annotations

import numbers

from dataclasses import dataclass, field
from typing import Callable, Dict, Tuple


@dataclass
class TaskSpec:
    priors: Dict[str, str]
    algorithm: Callable[[int, int], dict]     # (seed, population) -> algorithm config
    build: Callable                            # (population, device, seed, **kw) -> (task, pop, data)
    samples_per_trial: int                     # throughput unit (samples of one "trial")
    unit: str
    ckpt_factor: float = 4.0                   # checkpoint pool = factor x population
    # dimension names a user space may use (the task maps them onto member hyper-parameters)
    tunable: Tuple[str, ...] = ()
    required: Tuple[str, ...] = ("/lr",)       # must be in every space
    needs_fidelity: bool = False               # budgets come from the /steps fidelity only

    def check_space(self, space) -> None:
        """Refuse a user space this task cannot train: unknown names, missing required ones,
        a fidelity that is not ``/steps``."""
        names = list(space.keys())
        unknown = [n for n in names if n not in self.tunable]
        if unknown:
            raise ValueError(f"dimension(s) {unknown} are not hyper-parameters of this task; "
                             f"tunable: {sorted(self.tunable)}")
        missing = [n for n in self.required if n not in names]
        if missing:
            raise ValueError(f"the space must define {missing}")
        fids = [n for n, d in space.items() if d.type == "fidelity"]
        if any(n != "/steps" for n in fids):
            raise ValueError(f"the fidelity dimension must be /steps (optimizer steps), got {fids}")
        if self.needs_fidelity and not fids:
            raise ValueError("this task needs a /steps fidelity (its trials' budgets)")


def _max_width(priors, default):
    """Population slot width: the top of the /width prior (slots are sized for it)."""
    if "/width" not in priors:
        return default
    from ..space.builder import DimensionBuilder
    hi = DimensionBuilder().build("/width", priors["/width"]).interval()[1]
    width = int(hi)
    if width > 4096:
        raise ValueError(f"/width up to {width}: the population kernels are sized for <= 4096")
    return max(64, width)


def _max_batch(priors, default=128):
    """Population batch rows: the largest ``/batch_size`` the prior can draw (a categorical of
    multiples of 128, e.g. ``choices([128, 256, 512])``); members use their own first rows."""
    if "/batch_size" not in priors:
        return default
    from ..space.builder import DimensionBuilder
    dim = DimensionBuilder().build("/batch_size", priors["/batch_size"])
    values = getattr(dim, "categories", None)
    if dim.type != "categorical" or not values:
        raise ValueError("/batch_size must be a choices([...]) prior of multiples of 128")
    bad = [v for v in values if not isinstance(v, numbers.Real) or int(v) != v or int(v) % 128
           or int(v) < 128]
    if bad:
        raise ValueError(f"/batch_size choices must be multiples of 128, got {bad}")
    from ..ops.population import MAX_ROWS
    top = max(int(v) for v in values)
    if top > MAX_ROWS:
        raise ValueError(f"/batch_size up to {top}: the population kernels take <= {MAX_ROWS}")
    return top


def _mlp(population, device, seed, logreg=False, priors=None, state_dtype="bf16", **kw):
    from ..models.data import TeacherClassification
    from ..models.mlp import LOGREG_PRIORS, MLP_PRIORS, MLPSweepTask
    from ..ops.population import PopulationMLP
    priors = dict(priors or (LOGREG_PRIORS if logreg else MLP_PRIORS))
    max_width = 64 if logreg else _max_width(priors, 1024)
    batch = _max_batch(priors)
    task = MLPSweepTask(priors=priors, n_hidden=0 if logreg else 3,
                        in_features=2 if logreg else 784, num_classes=2 if logreg else 10,
                        width=64 if logreg else min(256, max_width), max_width=max_width)
    data = TeacherClassification(n_train=8192 if logreg else 60032, n_val=1024,
                                 in_features=task.in_features, num_classes=task.num_classes,
                                 teacher_hidden=4 if logreg else 128, seed=1234 + seed,
                                 batch_size=batch, device=device)
    on_gpu = str(device).startswith("cuda")
    pop = PopulationMLP(population, in_features=task.in_features, num_classes=task.num_classes,
                        n_hidden=task.n_hidden, max_width=task.max_width,
                        batch_size=batch, eval_batch=1024, device=device,
                        momentum_dtype="bf16" if (state_dtype == "bf16" and on_gpu) else "fp32")
    return task, pop, data


def _resnet(population, device, seed, batch_size=128, blocks=3, image_size=32, priors=None,
            **kw):
    from ..models.resnet import PopulationResNet, ResNetSweepTask, SyntheticCIFAR
    task = ResNetSweepTask(steps=kw.get("steps_per_trial", 390))
    if priors:
        task.priors = dict(priors)
    pop = PopulationResNet(population, batch_size=batch_size, device=device,
                           blocks_per_stage=blocks, image_size=image_size)
    data = SyntheticCIFAR(n_train=kw.get("n_train", 50048), n_val=1024, batch_size=batch_size,
                          seed=seed, device=device, image_size=image_size)
    return task, pop, data


def _lm(population, device, seed, preset="llama-125m", batch_size=8, seq_len=512, priors=None,
        state_dtype="bf16", **kw):
    import torch
    from ..models.llama import PRESETS, LM_PBT_PRIORS, LMSweepTask, PopulationLM, SyntheticLM
    cfg = PRESETS[preset]
    task = LMSweepTask(priors=dict(priors or LM_PBT_PRIORS), d_model=cfg.d_model)
    pop = PopulationLM(population, preset, batch_size=batch_size, seq_len=seq_len,
                       device=device, moment_dtype=(torch.bfloat16 if state_dtype == "bf16"
                                                    else torch.float32))
    data = SyntheticLM(cfg.vocab, seq_len, batch_size, n_tokens=kw.get("n_tokens", 1 << 22),
                       seed=seed, device=device)
    return task, pop, data


def _pbt(interval):
    return lambda seed, population: {"pbt": {"seed": seed, "population_size": population,
                                             "interval": interval,
                                             "min_forking_population": min(5, population)}}


TASKS: Dict[str, TaskSpec] = {
    "logreg": TaskSpec({"/lr": "loguniform(1e-3, 1.0)", "/weight_decay": "loguniform(1e-6, 1e-1)",
                        "/steps": "fidelity(64, 256, 2)"},
                       lambda seed, n: {"random": {"seed": seed}},
                       lambda p, d, s, **kw: _mlp(p, d, s, logreg=True, **kw), 8192,
                       "trials/s (1 trial = one pass over 8,192 samples)",
                       tunable=("/lr", "/weight_decay", "/momentum", "/steps", "/batch_size")),
    "mlp": TaskSpec({"/lr": "loguniform(1e-3, 1.0)",
                     "/width": "loguniform(64, 1024, discrete=True)",
                     "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(32, 2048, 4)"},
                    lambda seed, n: {"asha": {"seed": seed, "repetitions": float("inf")}},
                    _mlp, 60032, "trials/s (1 trial = 60,032 samples)",
                    tunable=("/lr", "/width", "/dropout", "/momentum", "/weight_decay",
                             "/steps", "/batch_size")),
    "resnet20": TaskSpec({"/lr": "loguniform(0.01, 0.5)", "/momentum": "uniform(0.5, 0.99)",
                          "/weight_decay": "loguniform(1e-5, 1e-2)"},
                         lambda seed, n: {"tpe": {"seed": seed, "n_initial_points": n}},
                         _resnet, 50048, "trials/s (1 trial = one CIFAR-sized epoch, 50,048 "
                                         "images)",
                         tunable=("/lr", "/momentum", "/weight_decay", "/steps")),
    "lm-125m": TaskSpec({"/lr": "loguniform(1e-4, 3e-3)",
                         "/weight_decay": "loguniform(1e-3, 0.3)", "/beta1": "uniform(0.8, 0.95)",
                         "/steps": "fidelity(200, 2000, 2)"},
                        _pbt(200), _lm, 8 * 512, "tokens/s", ckpt_factor=2.0,
                        tunable=("/lr", "/weight_decay", "/beta1", "/steps"),
                        needs_fidelity=True),
    "lm-tiny": TaskSpec({"/lr": "loguniform(1e-4, 3e-3)",
                         "/weight_decay": "loguniform(1e-3, 0.3)", "/beta1": "uniform(0.8, 0.95)",
                         "/steps": "fidelity(200, 2000, 2)"},
                        _pbt(200), lambda p, d, s, **kw: _lm(p, d, s, preset="tiny-2layer",
                                                             seq_len=256, **kw),
                        8 * 256, "tokens/s", ckpt_factor=2.0,
                        tunable=("/lr", "/weight_decay", "/beta1", "/steps"),
                        needs_fidelity=True),
}


def get(name: str) -> TaskSpec:
    if name not in TASKS:
        raise KeyError(f"unknown task {name!r}; choose from {sorted(TASKS)}")
    return TASKS[name]
