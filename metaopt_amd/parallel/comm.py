"""Process-group plumbing for the device data plane: one process per GPU, ``torch.distributed``
over RCCL (backend ``"nccl"`` on ROCm) on GPUs, ``gloo`` on CPU-only hosts (tests).

North-star collectives:
  * C1 ``all_gather_rows`` -- every rank gets every trial's metrics row (a few KB: latency-bound,
    so the population syncs every ``sync_every`` steps, one fused gather per sync);
  * C2 ``all_reduce_`` -- outer hyper-gradients (and intra-trial data-parallel gradients);
  * C4 ``send_tensor``/``recv_tensor`` and ``broadcast_`` -- PBT exploit weight copies (point to
    point over one xGMI link) and rank-0 decisions (C5).
With ``world_size == 1`` and no process group every call is a local no-op, so the same engine code
runs on one GPU without a rendezvous.

``MOPT_COMM_BACKEND=gloo`` runs GPU ranks over gloo instead (ranks may then share a GPU: the
device is ``LOCAL_RANK mod #GPUs``), staging GPU tensors through host memory -- a rehearsal of
the multi-rank engine on a one-GPU machine, not a production path.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int = 0, world_size: int = 1, local_rank: int = 0,
                 device: Optional[torch.device] = None, group=None):
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.device = device if device is not None else torch.device("cpu")
        self.group = group
        self.backend = dist.get_backend(group) if self.distributed else None

    @property
    def _host_staged(self) -> bool:
        """GPU tensors over a host-only backend (gloo rehearsal): copy through host memory."""
        return self.device.type == "cuda" and self.backend not in (None, "nccl")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    # -- collectives ----------------------------------------------------------------------------
    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """[n, m] per rank -> [world * n, m] on every rank (rank-major)."""
        if not self.distributed:
            return t
        t = t.contiguous()
        out = torch.empty((self.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.distributed:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.distributed:
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                   "min": dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=self.group)
        return t

    def all_reduce_mean_(self, t: torch.Tensor) -> torch.Tensor:
        self.all_reduce_(t, "sum")
        if self.distributed:
            t.div_(self.world_size)
        return t

    def send_tensor(self, t: torch.Tensor, dst: int) -> None:
        dist.send(t.contiguous(), dst=dst, group=self.group)

    def recv_tensor(self, t: torch.Tensor, src: int) -> torch.Tensor:
        dist.recv(t, src=src, group=self.group)
        return t

    def exchange(self, ops) -> None:
        """Batched point-to-point transfers: ``ops`` = [("send"|"recv", tensor, peer)].  One
        ``batch_isend_irecv`` group, so pairs of ranks sending to each other cannot deadlock."""
        if not ops:
            return
        if not self.distributed:
            raise RuntimeError("point-to-point exchange needs a process group")
        staged = []
        if self._host_staged:
            host_ops = []
            for kind, t, peer in ops:
                h = t.detach().cpu() if kind == "send" else torch.empty(t.shape, dtype=t.dtype)
                if kind == "recv":
                    staged.append((t, h))
                host_ops.append((kind, h, peer))
            ops = host_ops
        p2p = [dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer, group=self.group)
               for kind, t, peer in ops]
        for req in dist.batch_isend_irecv(p2p):
            req.wait()
        for t, h in staged:
            t.copy_(h)

    def barrier(self) -> None:
        if self.distributed:
            if self.device.type == "cuda" and self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index or 0])
            else:
                dist.barrier(group=self.group)

    def broadcast_object(self, obj, src: int = 0):
        if not self.distributed:
            return obj
        box: List = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    def all_gather_object(self, obj) -> list:
        """Every rank's ``obj`` (rank order) on every rank (small control-plane payloads)."""
        if not self.distributed:
            return [obj]
        out: List = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def max_float(self, value: float) -> float:
        """max over ranks of a host float (used for timing: the slowest rank sets the step)."""
        if not self.distributed:
            return float(value)
        t = torch.tensor([float(value)], dtype=torch.float64, device=self._coll_device())
        self.all_reduce_(t, "max")
        return float(t.item())

    def _coll_device(self):
        return self.device if self.device.type == "cuda" and not self._host_staged \
            else torch.device("cpu")


def init_from_env(backend: Optional[str] = None, timeout_s: int = 600) -> Comm:
    """Build a :class:`Comm` from torchrun's RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* variables.

    Selects ``cuda:LOCAL_RANK`` and the RCCL backend when GPUs are visible, gloo otherwise.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    backend = os.environ.get("MOPT_COMM_BACKEND") or backend
    if use_cuda:
        index = local_rank if backend in (None, "nccl") else local_rank % torch.cuda.device_count()
        torch.cuda.set_device(index)
        device = torch.device("cuda", index)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if use_cuda else "gloo")
        kwargs = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = device
        dist.init_process_group(**kwargs)
    return Comm(rank, world, local_rank, device)


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
