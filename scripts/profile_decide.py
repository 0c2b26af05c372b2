"""Host cost of the sweep's rank-0 decision step (ASHA observe/suggest, trial bookkeeping) on CPU.

Simulates ``WORLD`` ranks x 256 slots where every member reaches its budget on schedule, so the
decision path sees the same completion/placement volume as the GPU bench at that GPU count,
without a GPU:  ``WORLD=8 python scripts/profile_decide.py [--profile]``.
"""
import cProfile
import gc
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.io.experiment_builder import build_experiment  # noqa: E402
from metaopt_amd.models.mlp import MLP_PRIORS, MLPSweepTask  # noqa: E402
from metaopt_amd.storage.database import EphemeralDB  # noqa: E402
from metaopt_amd.storage.protocol import DocumentStorage  # noqa: E402
from metaopt_amd.worker.population_sweep import PopulationSweep  # noqa: E402


class _FakePop:
    """Just enough of PopulationMLP for the decision path."""

    def __init__(self, capacity):
        self.capacity = capacity
        self.device = __import__("torch").device("cpu")

    def alloc_ckpt_pool(self, n):
        pass


class _FakeComm:
    def __init__(self, world):
        self.world_size, self.rank, self.is_root = world, 0, True
        self.distributed = False
        import torch
        self.device = torch.device("cpu")

    def broadcast_object(self, obj, src=0):
        return obj

    def all_gather_object(self, obj):
        return [obj]


def _priors():
    """PRIORS=headline: bench.py's space (ASHA rungs 128 / 512 steps = 4 / 16 sync intervals: at
    8 ranks about 500 completions per sync); default: MLP_PRIORS (rung 0 = 32 steps, ONE sync
    interval: every rung-0 member finishes at every sync, about 1000 per sync -- the stress case)"""
    if os.environ.get("PRIORS", "stress") == "headline":
        sys.argv, argv = sys.argv[:1], sys.argv
        try:
            import bench
            return dict(bench.BENCH_PRIORS)
        finally:
            sys.argv = argv
    return dict(MLP_PRIORS)


def main(n_syncs=40, P=256, world=1, profile=False):
    priors = _priors()
    task = MLPSweepTask(priors=priors, max_width=1024)
    exp = build_experiment("decide-prof", priors=priors,
                           algorithms={"asha": ({"seed": 0, "unbounded": True}
                                                if os.environ.get("ASHA", "async") == "async"
                                                else {"seed": 0, "repetitions": float("inf")})},
                           storage=DocumentStorage(EphemeralDB()), pool_size=P)
    sw = PopulationSweep(_FakePop(P), task, data=None, comm=_FakeComm(world), experiment=exp,
                         sync_every=32, pipelined=False,
                         writer=os.environ.get("WRITER", "auto"))
    P = P * world                      # rows of the gathered status block
    rng = np.random.default_rng(0)
    steps = np.zeros(P)
    gathered = np.zeros((P, 9))
    gathered[:, 0] = -1
    gathered[:, 4] = -1
    assign = sw._decide(gathered)
    prof = cProfile.Profile() if profile else None
    t_total = t_rel = 0.0
    per_sync = []
    n_done = 0
    for _ in range(n_syncs):
        # apply: new/resumed members start from 0 (resume: from their checkpoint steps)
        for s in range(P):
            if assign[s, 0] in (1, 2):
                gathered[s, 0] = assign[s, 1]
                gathered[s, 2] = assign[s, 8]
                steps[s] = 0 if assign[s, 0] == 1 else gathered[s, 2] // 4
            elif assign[s, 0] == 3:
                gathered[s, 0] = -1
        steps += 32
        gathered[:, 1] = steps
        fin = (gathered[:, 0] >= 0) & (steps >= gathered[:, 2])
        n_done += int(fin.sum())
        gathered[:, 3] = 0
        gathered[:, 4] = np.where(fin, gathered[:, 0], -1)      # synchronous: results now
        gathered[:, 5] = rng.random(P)
        gathered[:, 6] = np.where(fin, rng.random(P), 0)
        gathered[:, 7] = 0.5
        gathered[:, 8] = 0
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        assign = sw._decide(gathered)
        if prof:
            prof.disable()
        per_sync.append(time.perf_counter() - t0)
        t_total += per_sync[-1]
        t1 = time.perf_counter()
        if not os.environ.get("NO_DRAIN"):
            sw._writer.drain_while(lambda: True)   # rank 0's share (inline: all of them)
        t_rel += time.perf_counter() - t1
        gc.freeze()                     # as PopulationSweep._sync does after every sync
    if hasattr(sw._writer, "_queue"):
        w = sw._writer
        print(f"at loop end: {w._queue.qsize()} messages not sent, "
              f"{w._handed - w._applied.value} ops not applied")
    t2 = time.perf_counter()
    if os.environ.get("NO_DRAIN") and profile:
        prof = cProfile.Profile()
        prof.enable()
        sw._writer.drain_all(4096)
        prof.disable()
    sw._writer.flush()
    t_flush = time.perf_counter() - t2
    n_ops = getattr(sw._writer, "_handed", None)
    kind = type(sw._writer).__name__
    sw.close()
    print(f"writer {kind}: final flush {1e3 * t_flush:.1f} ms"
          + (f", {n_ops / n_syncs:.0f} ops/sync handed over" if n_ops is not None else ""))
    print("phases ms/sync:", {k: round(1e3 * v / n_syncs, 2) for k, v in sw.timers.items()
                              if k.startswith("decide") or k.startswith("gc")})
    print(f"decide: {1e3 * t_total / n_syncs:.2f} ms/sync, writes {1e3 * t_rel / n_syncs:.2f} ms/sync, "
          f"{n_done / n_syncs:.1f} completions/sync; per sync p50 "
          f"{1e3 * float(np.median(per_sync)):.2f} ms, max {1e3 * max(per_sync):.2f} ms")
    if prof:
        pstats.Stats(prof).sort_stats(os.environ.get("SORT", "cumulative")).print_stats(30)


if __name__ == "__main__":
    if "--nogc" in sys.argv:
        import gc
        gc.disable()
    if os.environ.get("GC_T0"):
        gc.set_threshold(int(os.environ["GC_T0"]), 10, 10)
    main(n_syncs=int(os.environ.get("N_SYNCS", 40)), world=int(os.environ.get("WORLD", 1)),
         profile="--profile" in sys.argv)
