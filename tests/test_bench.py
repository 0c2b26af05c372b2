"""The headline bench's contract (bench.py): one JSON line, whole sync intervals in the timed
region, and ``--gpus N`` without torchrun spawning N ranks (gloo on this CPU host)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    # a one-interval bottom rung: trials complete within these few intervals
    args = (*args, "--fidelity", "1,4,4")
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert proc.returncode == 0, proc.stderr[-3000:]
    lines = [l for l in proc.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, proc.stdout
    return json.loads(lines[0])


def _check_contract(out, n, steps, warmup):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out, key
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == warmup
    assert out["scaling"] == "weak" and out["higher_is_better"] is True
    for key in ("model", "global_batch", "seq_len", "parallelism"):
        assert key in out["config"]
    # every timed step is one sync interval: the sweep loop (decide, C1, C5) ran in the timed
    # region and trials completed there
    assert out["timed_syncs"] == steps
    assert out["trials_completed"] > 0
    assert out["best_val_loss"] is not None
    for phase in ("decide", "c1_allgather", "c5_broadcast", "apply", "launch"):
        assert phase in out["host_ms_per_sync"], phase


def test_bench_one_rank_times_whole_sync_intervals():
    out = _run("--steps", "2", "--warmup", "1", "--population", "4", "--budget-intervals", "3")
    _check_contract(out, 1, 2, 1)
    assert out["budget"]["reached"] is True
    assert out["best_val_loss_at_budget"] is not None


def test_bench_spawns_ranks_without_torchrun():
    out = _run("--gpus", "2", "--steps", "1", "--warmup", "1", "--population", "4")
    _check_contract(out, 2, 1, 1)
    assert out["config"]["comm_backend"] == "gloo"
    assert out["config"]["parallelism"].startswith("dp2")
