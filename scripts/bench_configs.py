#!/usr/bin/env python
"""Throughput of the other BASELINE.json configurations (bench.py is the headline config 2).

    python scripts/bench_configs.py --config resnet20 --steps 40 --warmup 10
    python scripts/bench_configs.py --config lm-125m --population 8 --steps 20
    python scripts/bench_configs.py --config hyper --steps 3
    torchrun --nproc-per-node N scripts/bench_configs.py --config resnet20 ...

Each run is a real sweep: the task's search algorithm (TPE / PBT / random) on rank 0, device
populations on every rank, C1/C5 collectives every ``--sync-every`` steps (config 4: the C2
hypergradient all-reduce per outer step).  Data is synthetic, weights random-init.  Rank 0 prints
one JSON line.
"""
from __future__ import annotations

import argparse
import math
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEFAULT_POP = {"logreg": 64, "mlp": 256, "resnet20": 32, "lm-125m": 8, "lm-tiny": 16}
# the LM configs sync at the PBT interval (exploit / explore every 200 steps): the syncs between
# two generation boundaries would only read statistics back
DEFAULT_SYNC = {"logreg": 32, "mlp": 32, "resnet20": 30, "lm-125m": 200, "lm-tiny": 200}


def run_sweep(args, comm):
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import PopulationSweep
    from metaopt_amd.worker.tasks import get

    spec = get(args.config)
    P = args.population or DEFAULT_POP[args.config]
    sync_every = args.sync_every or DEFAULT_SYNC[args.config]
    kw = {}
    if args.config == "resnet20":
        kw["steps_per_trial"] = 390 // sync_every * sync_every
    task, pop, data = spec.build(P, comm.device, args.seed, **kw)
    exp = None
    if comm.is_root:
        exp = build_experiment(f"bench-{args.config}", priors=dict(task.priors),
                               algorithms=(spec.algorithm(args.seed, P * comm.world_size)
                                           if args.algo is None
                                           else {args.algo: {"seed": args.seed}}),
                               storage=DocumentStorage(EphemeralDB()),
                               pool_size=P * comm.world_size)
    sweep = PopulationSweep(pop, task, data, comm=comm, experiment=exp, sync_every=sync_every,
                            ckpt_capacity=max(4, int(spec.ckpt_factor * P)))
    on_gpu = comm.device.type == "cuda"
    if on_gpu and sweep._timeline is None:
        sweep._timeline = []   # GPU events at interval starts / syncs (per-generation report)
    sweep.start()
    for _ in range(args.warmup):
        sweep.step()
    sync(comm)
    s0, c0 = sweep.samples, sweep.completed
    sweep.timers.clear()
    sweep.n_syncs = 0
    if on_gpu:
        sweep._timeline = []
        sweep.copy_times(clear=True)
    marks = []                 # (host time after the sync, completed so far, global step)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sweep.step()
        if sweep.global_step % sync_every == 0:
            marks.append((time.perf_counter(), sweep.completed, sweep.global_step))
    if on_gpu:
        sweep._mark("interval")   # closes the last sync's GPU span
    sweep.flush()
    sync(comm)
    elapsed = comm.max_float(time.perf_counter() - t0)
    samples = torch.tensor([float(sweep.samples - s0)], dtype=torch.float64,
                           device=comm._coll_device())
    comm.all_reduce_(samples)
    samples = float(samples.item())
    # samples count sequences for the LMs: report tokens too
    per_sample = getattr(pop, "cfg", None)
    tokens = samples * per_sample.seq_len if per_sample is not None else None
    out = {"config": args.config, "n_gpus": comm.world_size, "population_per_gpu": P,
           "steps": args.steps, "warmup": args.warmup, "sync_every": sync_every,
           "ms_per_step": round(1e3 * elapsed / args.steps, 3),
           "samples_per_sec": round(samples / elapsed, 1),
           "trials_per_sec": round(samples / spec.samples_per_trial / elapsed, 4)
           if tokens is None else None,
           "tokens_per_sec": round(tokens / elapsed, 1) if tokens is not None else None,
           "completed_trials": sweep.completed - c0, "dtype": "bf16",
           "data": "synthetic",
           "params_per_trial": pop.n_params if isinstance(getattr(pop, "n_params", None), int)
           else None,
           "host_ms_per_sync": {k: round(1e3 * v / max(sweep.n_syncs, 1), 3)
                                for k, v in sweep.timers.items()}}
    if on_gpu:
        spans = _gpu_spans(sweep._timeline)
        out["gpu_ms_train_per_interval"] = _mean([a for a, _ in spans])
        out["gpu_ms_sync_per_interval"] = _mean([b for _, b in spans])
    if comm.is_root:
        summ = sweep.summary()
        out["best_val_loss"] = summ["best_val_loss"]
        # search quality over the run's completed trials, in completion order: the best at
        # 96 / 224 / all trials and the spread of every trial's validation loss
        vls = [h[2] for h in sweep.history if math.isfinite(h[2])]
        if vls:
            q = np.quantile(vls, [0.0, 0.1, 0.25, 0.5, 0.75, 1.0]).tolist()
            out["val_loss_quantiles"] = dict(zip(["min", "p10", "p25", "p50", "p75", "max"],
                                                 [round(v, 5) for v in q]))
            out["best_val_loss_at_trials"] = {str(n): round(min(vls[:n]), 5)
                                              for n in (32, 96, 224) if len(vls) >= n}
        out["algorithm"] = args.algo or next(iter(spec.algorithm(args.seed, P * comm.world_size)))
        inner = getattr(sweep.algorithm, "algorithm", sweep.algorithm)
        if hasattr(inner, "exploit_counts"):
            out.update(_pbt_report(sweep, inner, marks, t0, c0,
                                   spans if on_gpu else None,
                                   sweep.copy_times() if on_gpu else {}))
    sweep.close()
    return out


def _mean(v):
    return round(sum(v) / len(v), 3) if v else None


def _gpu_spans(timeline):
    """[(GPU ms of an interval's train steps, GPU ms from its sync to the next interval)] from
    the sweep's alternating interval / sync events (the sync span holds evaluation, checkpoint
    copies, member initialisation and any idle while the host decides)."""
    if not timeline:
        return []
    torch.cuda.synchronize()
    ev = [e for _, e, _ in timeline]
    kinds = [k for k, _, _ in timeline]
    out = []
    for i in range(len(kinds) - 2):
        if kinds[i] == "interval" and kinds[i + 1] == "sync" and kinds[i + 2] == "interval":
            out.append((ev[i].elapsed_time(ev[i + 1]), ev[i + 1].elapsed_time(ev[i + 2])))
    return out


def _pbt_report(sweep, algo, marks, t0, c0, spans, copies):
    """Per PBT generation boundary inside the timed window: wall ms of the generation (its
    training steps plus the boundary's evaluation, decision and exploit copies), the GPU split,
    the exploits / explores issued there and the generation's best validation loss."""
    counts = algo.exploit_counts()
    timeline = list(algo.timeline)
    best_by_budget = {}
    for _, _, vl, budget, _ in sweep.history:
        best_by_budget[budget] = min(vl, best_by_budget.get(budget, float("inf")))
    gens, prev_t, prev_c = [], t0, c0
    for i, (t, c, step) in enumerate(marks):
        row = {"end_step": step, "wall_ms": round(1e3 * (t - prev_t), 2),
               "completed": c - prev_c}
        if spans is not None and i < len(spans):
            row["gpu_train_ms"] = round(spans[i][0], 2)
            row["gpu_sync_ms"] = round(spans[i][1], 2)
        cp = copies.get(i, {})
        row["copy_ms"] = {k: round(v, 3) for k, v in cp.items()}
        if c - prev_c:
            # the members finishing here completed generation g; successors fork from it
            budgets = sorted({h[3] for h in sweep.history[prev_c:c]})   # one per completion
            g = timeline.index(budgets[-1]) if budgets and budgets[-1] in timeline else None
            if g is not None:
                row["generation"] = g
                row["exploits"], row["explores"] = counts.get(g, (0, 0))
                row["best_val_loss"] = round(best_by_budget.get(timeline[g], float("nan")), 5)
        gens.append(row)
        prev_t, prev_c = t, c
    bounds = [r for r in gens if "generation" in r]
    over = [100.0 * (r["wall_ms"] - r["gpu_train_ms"]) / r["wall_ms"]
            for r in bounds if r.get("gpu_train_ms")]
    copy_ms = [sum(r["copy_ms"].values()) for r in bounds]
    return {"pbt_interval": (timeline[1] - timeline[0]) if len(timeline) > 1 else None,
            "generations": gens,
            "exploit_rounds": sum(1 for r in bounds if r.get("exploits")),
            "exploits": sum(r.get("exploits", 0) for r in bounds),
            "explores": sum(r.get("explores", 0) for r in bounds),
            "ms_per_generation": _mean([r["wall_ms"] for r in bounds]),
            "exploit_copy_ms_per_generation": _mean(copy_ms),
            "generation_overhead_pct": _mean(over)}


def run_hyper(args, comm):
    from metaopt_amd.models.hyper import HypergradientSweep, HypergradLM
    from metaopt_amd.models.llama import SyntheticLM
    P = args.population or 8
    model = HypergradLM(P, "tiny-2layer", batch_size=4, seq_len=128, device=comm.device,
                        dp_comm=comm if getattr(args, "dp", False) else None)
    data = SyntheticLM(4096, 128, 4, n_tokens=1 << 20, seed=args.seed, device=comm.device)
    sweep = HypergradientSweep(model, data, comm=comm, inner_steps=args.inner_steps)
    for _ in range(args.warmup):
        sweep.step()
    sync(comm)
    t0 = time.perf_counter()
    hist = sweep.run(args.steps)
    sync(comm)
    elapsed = comm.max_float(time.perf_counter() - t0)
    inner = args.steps * args.inner_steps * P * comm.world_size
    return {"config": "hyper", "n_gpus": comm.world_size, "inner_runs_per_gpu": P,
            "outer_steps": args.steps, "inner_steps": args.inner_steps,
            "outer_steps_per_sec": round(args.steps / elapsed, 4),
            "inner_steps_per_sec": round(inner / elapsed, 2),
            "tokens_per_sec": round(inner * 4 * 128 / elapsed, 1),
            "final": hist[-1] if hist else None,
            "dtype": "bf16-operand MFMA GEMMs with fp32 accumulation; fp32 activations, "
                     "weights, tangents and optimizer state",
            "data": "synthetic"}


def sync(comm):
    if comm.device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if comm.device.type == "cuda":
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resnet20",
                    choices=["logreg", "mlp", "resnet20", "lm-125m", "lm-tiny", "hyper"])
    ap.add_argument("--dp", action="store_true",
                    help="hyper: intra-trial data parallelism (C3) instead of independent runs")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--population", type=int, default=None)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--sync-every", type=int, default=None)
    ap.add_argument("--inner-steps", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--algo", default=None,
                    help="override the config's search algorithm (e.g. random), default seed")
    args = ap.parse_args()
    if args.config != "hyper":
        every = args.sync_every or DEFAULT_SYNC[args.config]
        if args.steps % every or args.warmup % every:
            ap.error(f"--steps ({args.steps}) and --warmup ({args.warmup}) must be multiples of "
                     f"the sync interval ({every}): the timed window must hold whole intervals, "
                     "syncs included")
    from metaopt_amd.parallel.comm import init_from_env, shutdown
    comm = init_from_env()
    out = run_hyper(args, comm) if args.config == "hyper" else run_sweep(args, comm)
    if comm.is_root:
        print(json.dumps(out, default=str), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
