#!/usr/bin/env python
"""Headline benchmark: ASHA sweep of 4-layer MLPs, device populations, 1 process per GPU.

Metric (BASELINE.json): trials/sec for the whole node + best-loss@budget, 4-layer MLP sweep.

* One bench **step** is one *sync interval* of the population sweep: ``--sync-every`` (32)
  optimizer steps of every resident trial (HIP kernels), followed by the sync -- validation of the
  trials that reached their budget, C1 metric all-gather, ASHA observe/suggest on rank 0, C5
  assignment broadcast, (re)initialisation of new members and checkpoint-resume of promoted ones.
  Every timed step therefore contains the whole sweep loop, whatever ``--steps`` is.
* ``value`` counts *epoch-equivalent* trials: 60,032 samples (469 steps x 128) through a 4-layer
  MLP 784-w-w-w-10 -- the unit of the reference's MNIST tutorial sweep (5 trials in 49.75 s =
  0.1005 trials/s, reference docs/src/user/pytorch.rst:131-136).  The JSON also reports the
  ASHA trials actually completed (one trial document per rung evaluation, as in the reference's
  ASHA) per second, and the best validation loss at a fixed budget of ``--budget-intervals``
  sync intervals from the start of the sweep (stated in the JSON).
* ASHA is the asynchronous (unbounded) algorithm of Li et al. over ``fidelity(128, 512, 4)``
  optimizer steps (rungs 128/512; the top rung is 65,536 samples ~ one MNIST epoch), so complete
  ladders fit in the driver's short run.  Chosen on the GPU (profiles/r4/algo_*.json, one box):
  at 24 intervals it reaches a lower best loss than random search (1.1456 vs 1.1544) at random
  search's throughput, where the reference's bounded brackets lost to random (1.1633).
* Weak scaling: every GPU holds ``--population`` (256) trials.

``python bench.py --gpus N --steps K --warmup W``.  Under torchrun (WORLD_SIZE set) every process
is one rank.  Without it and ``N > 1`` this process is only a launcher: it starts N rank processes
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1) without touching the GPU itself, and when the
machine has fewer than N GPUs the ranks share them over gloo (a rehearsal, flagged in the JSON).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "trials/sec (whole node) + best-loss@budget, 4-layer MLP sweep at 1/2/4/8 MI355X"
BASELINE_TRIALS_PER_SEC = 5.0 / 49.751548  # reference MNIST tutorial sweep
SAMPLES_PER_TRIAL = 60032                   # one epoch-equivalent of MNIST (469 x 128)
BENCH_PRIORS = {
    "/lr": "loguniform(1e-3, 1.0)",
    "/width": "loguniform(64, 1024, discrete=True)",
    "/dropout": "uniform(0, 0.5)",
    "/steps": "fidelity(128, 512, 4)",   # replaced from --fidelity and --sync-every
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed sync intervals")
    ap.add_argument("--warmup", type=int, default=5, help="untimed sync intervals")
    ap.add_argument("--population", type=int, default=256, help="trials per GPU")
    ap.add_argument("--max-width", type=int, default=1024)
    ap.add_argument("--sync-every", type=int, default=32,
                    help="optimizer steps per sync interval (= one bench step)")
    ap.add_argument("--budget-intervals", type=int, default=24,
                    help="best-loss@budget: best validation loss of the trials finished within "
                         "this many sync intervals from the start of the sweep")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--algo", default="asha", choices=["asha", "random", "tpe"])
    ap.add_argument("--asha-mode", default="async", choices=["async", "bounded"],
                    help="async: Li et al.'s unbounded asynchronous ASHA; bounded: the "
                         "reference's bracket semantics repeated (repetitions=inf)")
    ap.add_argument("--fidelity", default="4,16,4",
                    help="ASHA fidelity 'min,max,base' in sync intervals (steps = x sync_every)")
    ap.add_argument("--momentum-dtype", default="bf16", choices=["fp32", "bf16"],
                    help="SGD momentum buffer precision (weights: f32 master + bf16 copy)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------- launcher
def launch(n: int, argv) -> int:
    """Start ``n`` rank processes of this script and wait for them (this process never touches
    the GPU; see metaopt_amd/parallel/launch.py)."""
    from metaopt_amd.parallel.launch import spawn
    return spawn(n, [os.path.abspath(__file__), *argv])


# ---------------------------------------------------------------------------------- one rank
def run_rank(args) -> None:
    import torch

    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.data import TeacherClassification
    from metaopt_amd.models.mlp import MLPSweepTask
    from metaopt_amd.ops.population import PopulationMLP
    from metaopt_amd.parallel.comm import init_from_env, shutdown
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import PopulationSweep

    comm = init_from_env()
    on_gpu = comm.device.type == "cuda"
    if not on_gpu:   # CPU ranks share the host's cores
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", 0))
                              or max(1, (os.cpu_count() or 1) // comm.world_size))
    P = args.population if on_gpu else min(args.population, 8)
    max_width = args.max_width if on_gpu else min(args.max_width, 256)
    S = args.sync_every
    priors = dict(BENCH_PRIORS)
    f_min, f_max, f_base = (int(v) for v in args.fidelity.split(","))
    priors["/steps"] = f"fidelity({f_min * S}, {f_max * S}, {f_base})"
    if not on_gpu:  # CPU smoke configuration (the GPU path is the measured one)
        priors["/width"] = f"loguniform(64, {max_width}, discrete=True)"
    task = MLPSweepTask(priors=priors, max_width=max_width)

    experiment = None
    if comm.is_root:
        storage = DocumentStorage(EphemeralDB())
        asha_cfg = ({"seed": args.seed, "unbounded": True} if args.asha_mode == "async" else
                    {"seed": args.seed, "repetitions": float("inf")})
        algo = {"asha": {"asha": asha_cfg},
                "random": {"random": {"seed": args.seed}},
                "tpe": {"tpe": {"seed": args.seed, "n_initial_points": P}}}[args.algo]
        experiment = build_experiment("bench-mlp-sweep", priors=priors, algorithms=algo,
                                      storage=storage, pool_size=P)
    data = TeacherClassification(n_train=SAMPLES_PER_TRIAL if on_gpu else 4096, n_val=1024,
                                 batch_size=128, seed=1234 + args.seed, device=comm.device)
    pop = PopulationMLP(P, max_width=max_width, eval_batch=1024, device=comm.device,
                        momentum_dtype=args.momentum_dtype)
    # staggered start (populations over 512 slots): finished inside the untimed warm-up
    stagger = min(4, max(1, -(-comm.world_size * P // 512)), max(1, args.warmup - 1))
    sweep = PopulationSweep(pop, task, data, comm=comm, experiment=experiment,
                            sync_every=S, ckpt_capacity=4 * P, stagger=stagger)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def interval():
        sweep.run_interval()     # S optimizer steps queued in one host call, then the sync

    sweep.start()
    for _ in range(args.warmup):
        interval()
    sweep.flush()
    sync()
    comm.barrier()
    sync()
    sweep.gpu_timeline(clear=True)
    s0, c0, n0 = sweep.samples, sweep.completed, sweep.n_syncs
    sweep.timers.clear()
    sweep.n_syncs = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        interval()
    sweep.flush()            # deferred storage writes belong to the timed work
    sync()
    comm.barrier()
    sync()
    elapsed = comm.max_float(time.perf_counter() - t0)
    local = torch.tensor([float(sweep.samples - s0)], dtype=torch.float64,
                         device=comm._coll_device())
    comm.all_reduce_(local)
    samples = float(local.item())
    n_syncs = sweep.n_syncs
    completed = sweep.completed - c0     # rank 0 records every trial of every rank
    trials_per_sec = samples / SAMPLES_PER_TRIAL / elapsed
    if comm.is_root:
        summ = sweep.summary()
        budget_steps = args.budget_intervals * S
        at_budget = sweep.best_within(budget_steps)
        reached = sweep.global_step >= budget_steps
        rehearsal = os.environ.get("MOPT_BENCH_REHEARSAL") == "1"
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
                "algorithm": args.algo if args.algo != "asha" else f"asha ({args.asha_mode})",
                "population_per_gpu": P,
                "global_batch": 128 * P * comm.world_size,
                "seq_len": None,
                "parallelism": f"dp{comm.world_size} (trial-parallel populations)",
                "search_space": priors,
                "step": f"one sync interval = {S} optimizer steps of every trial + the sync "
                        "(validation, C1 all-gather, decide, C5 broadcast, member init/resume)",
                "backend": pop.backend,
                "stream_groups": pop.n_streams,
                # each step's first-layer backward + update fused with the next step's
                # first-layer forward (bit-identical to separate launches; MOPT_FUSE0=0 off)
                "fused_first_layer": bool(getattr(pop, "fuse_first_layer", False)),
                "optimizer_state": f"f32 master weights + bf16 copy, {args.momentum_dtype} "
                                   "SGD momentum",
                "comm_backend": comm.backend or "none",
                "rehearsal_ranks_share_gpus": rehearsal,
                # syncs the first fill is spread over (populations over 512 slots: the members'
                # budgets then end in different syncs, rank 0's decision work stays even)
                "staggered_start_syncs": sweep.stagger,
            },
            "timed_syncs": n_syncs,
            "trials_completed": completed,
            "trials_completed_per_sec": round(completed / elapsed, 2),
            "trials_completed_before_timing": c0,
            "best_val_loss": None if not math.isfinite(summ["best_val_loss"])
            else round(summ["best_val_loss"], 5),
            "best_params": summ["best_params"],
            "best_val_loss_at_budget": (round(at_budget[0], 5)
                                        if reached and math.isfinite(at_budget[0]) else None),
            "budget": {"sync_intervals": args.budget_intervals,
                       "optimizer_steps_per_slot": budget_steps,
                       "samples_per_gpu": budget_steps * 128 * P,
                       "trials_finished_within": at_budget[1],
                       "reached": reached},
            # best-loss at several budgets (sync intervals from the start of the sweep)
            "best_val_loss_at_intervals": {
                str(n): (round(sweep.best_within(n * S)[0], 5)
                         if sweep.global_step >= n * S and math.isfinite(sweep.best_within(n * S)[0])
                         else None) for n in (12, 24, 48)},
            "samples_per_sec": round(samples / elapsed, 1),
            "host_ms_per_sync": summ["host_ms_per_sync"],
            **({"gpu_timeline": sweep.gpu_timeline()} if os.environ.get("MOPT_GPU_TIMELINE")
               else {}),
            "warmup_syncs": n0,
        }
        print(json.dumps(out), flush=True)
    shutdown()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, argv))
    run_rank(args)


if __name__ == "__main__":
    main()
