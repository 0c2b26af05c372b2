#!/usr/bin/env python
"""Headline benchmark: ASHA sweep of 4-layer MLPs, device populations, 1 process per GPU.

Metric (BASELINE.json): trials/sec for the whole node + best-loss@budget, 4-layer MLP sweep.
  * one *trial* = one epoch-equivalent (60,032 samples, 469 steps x 128) of a 4-layer MLP
    784-w-w-w-10 (w ~ loguniform(64, 1024)), SGD-momentum, dropout, bf16 compute -- the unit of
    the reference's MNIST tutorial sweep (5 trials in 49.75 s = 0.1005 trials/s,
    reference docs/src/user/pytorch.rst:131-136);
  * the timed region is the whole sweep loop: population train steps (HIP kernels), validation
    of finished trials, C1 metric all-gather, ASHA decisions on rank 0, C5 assignment broadcast,
    member (re)initialisation and checkpoint-resume of promoted trials;
  * weak scaling: every GPU holds ``--population`` (256) trials.

``python bench.py --gpus N --steps K --warmup W``; for N > 1 launch with torchrun (one rank per
GPU).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "trials/sec (whole node) + best-loss@budget, 4-layer MLP sweep at 1/2/4/8 MI355X"
BASELINE_TRIALS_PER_SEC = 5.0 / 49.751548  # reference MNIST tutorial sweep
SAMPLES_PER_TRIAL = 60032                   # one epoch-equivalent of MNIST (469 x 128)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=320)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--population", type=int, default=256)
    ap.add_argument("--max-width", type=int, default=1024)
    ap.add_argument("--sync-every", type=int, default=32,
                    help="population sync interval (steps); budgets are multiples of it")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--algo", default="asha", choices=["asha", "random", "tpe"])
    args = ap.parse_args(argv)

    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.data import TeacherClassification
    from metaopt_amd.models.mlp import MLP_PRIORS, MLPSweepTask
    from metaopt_amd.ops.population import PopulationMLP
    from metaopt_amd.parallel.comm import init_from_env, shutdown
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import PopulationSweep

    comm = init_from_env()
    on_gpu = comm.device.type == "cuda"
    P = args.population if on_gpu else min(args.population, 8)
    max_width = args.max_width if on_gpu else min(args.max_width, 256)
    priors = dict(MLP_PRIORS)
    if not on_gpu:  # CPU smoke configuration (the GPU path is the measured one)
        priors["/width"] = f"loguniform(64, {max_width}, discrete=True)"
    task = MLPSweepTask(priors=priors, max_width=max_width)

    experiment = None
    if comm.is_root:
        storage = DocumentStorage(EphemeralDB())
        algo = {"asha": {"asha": {"seed": args.seed, "repetitions": float("inf")}},
                "random": {"random": {"seed": args.seed}},
                "tpe": {"tpe": {"seed": args.seed, "n_initial_points": P}}}[args.algo]
        experiment = build_experiment("bench-mlp-sweep", priors=priors, algorithms=algo,
                                      storage=storage, pool_size=P)
    data = TeacherClassification(n_train=SAMPLES_PER_TRIAL if on_gpu else 4096, n_val=1024,
                                 batch_size=128, seed=1234 + args.seed, device=comm.device)
    pop = PopulationMLP(P, max_width=max_width, eval_batch=1024, device=comm.device)
    sweep = PopulationSweep(pop, task, data, comm=comm, experiment=experiment,
                            sync_every=args.sync_every, ckpt_capacity=4 * P)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    sweep.start()
    for _ in range(args.warmup):
        sweep.step()
    sync()
    comm.barrier()
    sync()
    s0, c0 = sweep.samples, sweep.completed
    sweep.timers.clear()
    sweep.n_syncs = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sweep.step()
    sweep.flush()            # deferred storage writes belong to the timed work
    sync()
    comm.barrier()
    sync()
    elapsed = comm.max_float(time.perf_counter() - t0)
    local_samples = torch.tensor([float(sweep.samples - s0)], dtype=torch.float64,
                                 device=comm._coll_device())
    comm.all_reduce_(local_samples)
    samples = float(local_samples.item())
    completed = sweep.completed - c0
    trials_per_sec = samples / SAMPLES_PER_TRIAL / elapsed
    if comm.is_root:
        summ = sweep.summary()
        out = {
            "metric": METRIC,
            "value": round(trials_per_sec, 3),
            "unit": "trials/s (1 trial = 1 epoch-equivalent: 60,032 samples through a 4-layer "
                    "MLP, fwd+bwd+SGD)",
            "n_gpus": comm.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(trials_per_sec / BASELINE_TRIALS_PER_SEC, 2),
            "dtype": "bf16",
            "data": "synthetic (teacher-labelled MNIST-shaped 784->10, random-init weights)",
            "config": {
                "model": "4-layer MLP 784-w-w-w-10, w~loguniform(64,1024), dropout, SGD-momentum",
                "algorithm": args.algo,
                "population_per_gpu": P,
                "global_batch": 128 * P * comm.world_size,
                "seq_len": None,
                "parallelism": f"dp{comm.world_size} (trial-parallel populations)",
                "trial_budget": "ASHA fidelity(32, 2048, 4) steps; throughput counted in "
                                "epoch-equivalents",
                "sync_every": args.sync_every,
                "backend": pop.backend,
            },
            "asha_trials_completed": completed,
            "asha_trials_completed_per_sec": round(completed / elapsed, 2),
            "best_val_loss": None if not math.isfinite(summ["best_val_loss"])
            else round(summ["best_val_loss"], 5),
            "best_params": summ["best_params"],
            "samples_per_sec": round(samples / elapsed, 1),
            "host_ms_per_sync": summ["host_ms_per_sync"],
        }
        print(json.dumps(out), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
