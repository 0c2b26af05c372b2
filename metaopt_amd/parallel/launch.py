"""Single-node launcher: one rank process per GPU (``mopt sweep --gpus N``, ``bench.py --gpus N``).

The launching process never initialises HIP (it only counts devices, which does not on this
image) and starts the ranks as child processes -- it never ``exec``s into one.  Ranks get
``RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT`` and
rendezvous through :func:`metaopt_amd.parallel.comm.init_from_env` (RCCL on GPUs).  When the
host has fewer GPUs than ranks (a rehearsal on a one-GPU box) or none (CPU tests) the ranks use
gloo and share what there is (``MOPT_COMM_BACKEND=gloo``).  If one rank fails the others are
terminated (they would otherwise wait in a collective forever) and its exit code is returned.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(n: int, base: Optional[dict] = None, port: Optional[int] = None) -> dict:
    """Environment shared by the ``n`` ranks (RANK / LOCAL_RANK are added per rank)."""
    import torch
    env = dict(os.environ if base is None else base)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port or free_port()),
               WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    n_dev = torch.cuda.device_count()
    if n_dev < n:
        env["MOPT_COMM_BACKEND"] = "gloo"
        if n_dev > 0:
            env["MOPT_BENCH_REHEARSAL"] = "1"    # ranks share the GPUs
    return env


def spawn(n: int, argv: Sequence[str], env: Optional[dict] = None,
          poll_s: float = 0.05) -> int:
    """Run ``[python] + argv`` as ``n`` ranks and wait; returns the first failing exit code."""
    env = rank_env(n) if env is None else env
    procs: List[subprocess.Popen] = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, *argv],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r))))
    code = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                rc = p.poll()
                if rc is None:
                    continue
                pending.remove(p)
                if rc != 0 and code == 0:
                    code = rc
                    for q in pending:        # the survivors would hang in a collective
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return code
