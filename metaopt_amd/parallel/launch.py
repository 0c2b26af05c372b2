"""Single-node launcher: one rank process per GPU (``mopt sweep --gpus N``, ``bench.py --gpus N``).

The launching process never touches HIP: it counts the GPUs from the kernel driver's KFD topology
in sysfs and the visible-devices variables (:func:`visible_gpu_count`), and starts the ranks as
child processes -- it never ``exec``s into one.  Ranks get
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


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
_VISIBLE_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


DRI_DIR = "/dev/dri"


def _kfd_gpu_count(root: str = KFD_NODES, dri: str = DRI_DIR) -> int:
    """GPU agents in the KFD topology that this process can open: nodes whose ``properties``
    report SIMDs (CPU nodes have ``simd_count 0``) and whose render node
    ``/dev/dri/renderD<drm_render_minor>`` exists and is read/writable -- sysfs lists every GPU
    of the host even in a container given only some render nodes.  0 when the driver is
    absent."""
    try:
        nodes = os.listdir(root)
    except OSError:
        return 0
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(root, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if line.strip())
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        minor = props.get("drm_render_minor", "").strip()
        if minor and int(minor) > 0:
            dev = os.path.join(dri, f"renderD{int(minor)}")
            if not os.access(dev, os.R_OK | os.W_OK):
                continue
        n += 1
    return n


def visible_gpu_count(env: Optional[dict] = None, root: str = KFD_NODES,
                      dri: str = DRI_DIR) -> int:
    """GPUs a child process will see, without initialising HIP in this one: the KFD topology's
    accessible GPU count, narrowed by ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` /
    ``CUDA_VISIBLE_DEVICES`` (each applied in that order, as the runtime does).
    ``MOPT_GPU_COUNT`` overrides the topology count."""
    env = os.environ if env is None else env
    forced = env.get("MOPT_GPU_COUNT")
    n = int(forced) if forced not in (None, "") else _kfd_gpu_count(root, dri)
    for var in _VISIBLE_VARS:
        val = env.get(var)
        if val is None:
            continue
        ids = [v for v in val.split(",") if v.strip()]
        if not ids or ids[0].strip() == "-1":
            return 0
        n = min(n, len(ids))
    return n


def rank_env(n: int, base: Optional[dict] = None, port: Optional[int] = None) -> dict:
    """Environment shared by the ``n`` ranks (RANK / LOCAL_RANK are added per rank)."""
    env = dict(os.environ if base is None else base)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port or free_port()),
               WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    n_dev = visible_gpu_count(env)
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
