"""Populations of same-architecture trials on flat parameter buffers (the LM and CNN paths).

A :class:`FlatPopulation` keeps ``capacity`` trials of ONE architecture on a device.  Every
parameter tensor is stacked over the population (``[P, ...]``) and lives in flat buffers:

* ``p16`` -- bf16 working weights; the autograd leaves are views of it, and their ``.grad`` is
  pre-bound to views of the flat bf16 gradient ``g16`` (autograd accumulates in place, so the
  whole population's gradient is one contiguous buffer);
* the f32 master weights -- on the GPU split (csrc/common.h): ``p16`` is their high half and
  ``plo`` (int16) the low half, so the master costs 2 bytes beyond the working copy; on the CPU
  reference backend a plain f32 ``p32`` -- and ``m``/``v``, the optimizer state; one fused
  kernel updates every tensor of every trial with per-trial hyper-parameters (AdamW: K6,
  SGD-momentum: K5; 22 bytes per parameter and step for AdamW with the bf16 first moment);
* ``aux`` -- per-trial non-parameter state (e.g. BatchNorm running statistics), checkpointed
  with the weights.

Subclasses define ``param_specs()`` / ``aux_size()`` and ``_loss(x, y, train)`` (per-trial loss
sums, optionally per-trial #correct).  The member interface -- ``set_member``,
``update_hparams``, ``remove_member``, ``train_step``, ``evaluate_async`` / ``eval_result``,
``save_states`` / ``load_states`` (one batched copy kernel), ``pack_state`` / ``unpack_state``
(C4 transfers) -- is what :class:`~metaopt_amd.worker.population_sweep.PopulationSweep` drives.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import _lib
from ..ops import lm as ops
from ..ops.population import MemberConfig, device_busy


INIT_SEG_DTYPE = np.dtype([("p32", "<u8"), ("p16", "<u8"), ("m", "<u8"), ("v", "<u8"),
                           ("n", "<i8"), ("kind", "<i4"), ("val", "<f4"), ("seed", "<u4"),
                           ("tag", "<u4"), ("m16", "<i4"), ("split", "<i4")])
assert INIT_SEG_DTYPE.itemsize == 64
_CHUNK = 4096
_CHUNK_DTYPE = np.dtype([("desc", "<i4"), ("pad", "<i4"), ("start", "<i8")])
_lib.register_signatures({
    "mopt_flat_init": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
                       ctypes.c_int),
})


class FlatPopulation:
    optimizer = "adamw"            # or "sgd"
    moment_dtype = torch.float32   # AdamW first-moment storage (bf16: see lm_ops.hip adamw)
    secondary = "acc"              # eval_result's second array: "acc" or "ppl"

    def __init__(self, capacity: int, device="cuda", max_grad_norm: float = 0.0,
                 use_graph: bool = True):
        self.device = torch.device(device)
        self.use_graph = bool(use_graph)
        self._graph = None
        self.backend = "hip" if self.device.type == "cuda" else "torch"
        self.capacity = P = int(capacity)
        self.max_grad_norm = float(max_grad_norm)
        self.specs = self.param_specs()
        self.segments = []
        off = 0
        for name, shape, _ in self.specs:
            n = int(np.prod(shape))
            if n % 8:
                raise ValueError(f"parameter {name}: per-trial size {n} must be a multiple of 8 "
                                 "(the fused optimizer moves 8 elements per lane)")
            self.segments.append((off, n))
            off += P * n
        self.n_flat = off
        dev = self.device
        # split master on the GPU (the fused optimizer joins / splits it in registers)
        self.split = self.device.type == "cuda"
        self.plo = torch.zeros(off, dtype=torch.int16, device=dev) if self.split else None
        self.p32 = None if self.split else torch.zeros(off, dtype=torch.float32, device=dev)
        self.p16 = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        self.g16 = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        self.m = torch.zeros(off, dtype=self.moment_dtype if self.optimizer == "adamw"
                             else torch.float32, device=dev)
        self.v = (torch.zeros(off, dtype=torch.float32, device=dev) if self.optimizer == "adamw"
                  else torch.zeros(0, dtype=torch.float32, device=dev))
        # per-trial non-parameter state, segment-major like the parameters: A[name] is [P, n]
        self.aux_segments, aoff = [], 0
        for name, n in self.aux_specs():
            self.aux_segments.append((name, aoff, int(n)))
            aoff += P * int(n)
        self.n_aux = sum(n for _, _, n in self.aux_segments)
        self.aux = torch.zeros(max(aoff, 4), dtype=torch.float32, device=dev)
        self.A = {name: self.aux[o:o + P * n].view(P, n) for name, o, n in self.aux_segments}
        self.W: Dict[str, torch.Tensor] = {}
        for (name, shape, _), (o, n) in zip(self.specs, self.segments):
            leaf = self.p16[o:o + P * n].view(P, *shape)
            leaf.requires_grad_(True)
            leaf.grad = self.g16[o:o + P * n].view(P, *shape)
            self.W[name] = leaf
        # gradients the HIP kernels overwrite every step (straight into the .grad views) need no
        # zeroing; the rest (autograd-accumulated) is zeroed per step, contiguous runs merged
        direct = self.direct_grads() if self.device.type == "cuda" else set()
        self._zero_runs = []
        for (name, _, _), (o, n) in zip(self.specs, self.segments):
            if name in direct:
                continue
            if self._zero_runs and self._zero_runs[-1][1] == o:
                self._zero_runs[-1][1] = o + P * n
            else:
                self._zero_runs.append([o, o + P * n])
        self.opt = ops.FlatOptimizer(self.segments, P, dev, kind=self.optimizer)
        self.hp = np.zeros(P, dtype=[("t", "<i4")])
        self.opt_hp = np.zeros(P, dtype=ops.LM_HP_DTYPE)
        self.members: List[Optional[MemberConfig]] = [None] * P
        self.stats = torch.zeros(4 * P, dtype=torch.float32, device=dev)
        self._ck = None
        self._ck_aux = None

    # ------------------------------------------------------------------ subclass hooks
    def param_specs(self):
        """[(name, per-trial shape, init)]; init = ('normal', std) | ('ones',) | ('zeros',) |
        ('kaiming', fan_in)."""
        raise NotImplementedError

    def direct_grads(self):
        """Names of the parameters whose gradient the HIP backward writes in full every step
        (no zeroing, no accumulation); default: none."""
        return set()

    def aux_specs(self):
        """[(name, per-trial numel)] of the non-parameter state (checkpointed with the weights)."""
        return []

    def init_aux(self, slot: int) -> None:
        pass

    def _loss(self, x, y, train: bool):
        """Per-trial loss sums [P] (and optionally #correct [P]) of batch (x, y)."""
        raise NotImplementedError

    def rows_per_batch(self, x) -> int:
        return int(x.shape[0])

    # ------------------------------------------------------------------ members
    @property
    def n_params(self) -> int:
        return sum(n for _, n in self.segments)

    def active_slots(self):
        return [s for s, m in enumerate(self.members) if m is not None]

    def _write_hp(self, slot, cfg: MemberConfig, t: int):
        self.hp[slot]["t"] = t
        self.opt_hp[slot] = (cfg.lr, cfg.momentum, cfg.beta2, cfg.eps, cfg.weight_decay,
                             self.max_grad_norm, t, 0)

    def _slices(self, slot):
        return [slice(o + slot * n, o + (slot + 1) * n) for o, n in self.segments]

    def _aux_slices(self, slot):
        return [slice(o + slot * n, o + (slot + 1) * n) for _, o, n in self.aux_segments]

    def _aux_of(self, slot) -> torch.Tensor:
        sl = self._aux_slices(slot)
        return torch.cat([self.aux[x] for x in sl]) if sl else torch.zeros(0, device=self.device)

    def _set_aux(self, slot, flat) -> None:
        o = 0
        for x in self._aux_slices(slot):
            n = x.stop - x.start
            self.aux[x] = flat[o:o + n]
            o += n

    @torch.no_grad()
    def set_member(self, slot: int, cfg: MemberConfig, init: bool = True) -> None:
        self.members[slot] = cfg
        self._write_hp(slot, cfg, 0)
        if not init:
            return
        if self.device.type == "cuda" and _lib.available():
            self._init_member_hip(slot, int(cfg.seed) & 0x7FFFFFFF)
            return
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(cfg.seed) & 0x7FFFFFFF)
        for (name, shape, init_), sl in zip(self.specs, self._slices(slot)):
            dst = self.p32[sl] if not self.split else torch.empty(
                sl.stop - sl.start, dtype=torch.float32, device=self.device)
            kind = init_[0]
            if kind == "ones":
                dst.fill_(1.0)
            elif kind == "zeros":
                dst.zero_()
            elif kind == "normal":
                dst.normal_(0.0, init_[1], generator=gen)
            elif kind == "kaiming":
                dst.normal_(0.0, (2.0 / init_[1]) ** 0.5, generator=gen)
            else:
                raise ValueError(f"unknown init {init_}")
            self._set_master_slice(sl, dst)
            self.m[sl].zero_()
            if self.v.numel():
                self.v[sl].zero_()
        self.init_aux(slot)

    def aux_fill_specs(self):
        """[(aux name, offset, length, value)] constant fills that initialise a member's
        non-parameter state on the GPU path (one launch with the parameters); None: call
        ``init_aux`` instead."""
        return None

    def _init_member_hip(self, slot: int, seed: int) -> None:
        """Parameters (constant / N(0, std) from the counter-based RNG, tag = tensor index),
        bf16 copies, zeroed moments and the constant fills of the non-parameter state in ONE
        ``mopt_flat_init`` launch (csrc/copy_kernels.hip)."""
        segs = []
        m16 = self.m.dtype == torch.bfloat16
        mbuf = self.master_buf
        p32, p16, mm = mbuf.data_ptr(), self.p16.data_ptr(), self.m.data_ptr()
        v = self.v.data_ptr() if self.v.numel() else 0
        e32, e16, em = mbuf.element_size(), self.p16.element_size(), self.m.element_size()
        for i, ((name, shape, init_), (o, n)) in enumerate(zip(self.specs, self.segments)):
            start = o + slot * n
            kind = init_[0]
            if kind == "ones":
                k, val = 0, 1.0
            elif kind == "zeros":
                k, val = 0, 0.0
            elif kind == "normal":
                k, val = 1, float(init_[1])
            elif kind == "kaiming":
                k, val = 1, float((2.0 / init_[1]) ** 0.5)
            else:
                raise ValueError(f"unknown init {init_}")
            segs.append((p32 + start * e32, p16 + start * e16, mm + start * em,
                         v + start * 4 if v else 0, n, k, val, seed, 0x3000 + i, int(m16),
                         int(self.split)))
        fills = self.aux_fill_specs()
        if fills is not None:
            a32 = self.aux.data_ptr()
            offs = {name: (o, n) for name, o, n in self.aux_segments}
            for name, off, length, val in fills:
                o, n = offs[name]
                segs.append((a32 + (o + slot * n + off) * 4, 0, 0, 0, length, 0, float(val), 0,
                             0, 0, 0))
        arr = np.array(segs, dtype=INIT_SEG_DTYPE)
        counts = (arr["n"] + _CHUNK - 1) // _CHUNK
        chunks = np.zeros(int(counts.sum()), dtype=_CHUNK_DTYPE)
        chunks["desc"] = np.repeat(np.arange(len(arr), dtype=np.int32), counts)
        first = np.concatenate([[0], np.cumsum(counts)[:-1]])
        chunks["start"] = (np.arange(len(chunks)) - np.repeat(first, counts)) * _CHUNK
        d = _lib.upload_bytes(arr, self.device)
        c = _lib.upload_bytes(chunks, self.device)
        _lib.check(_lib.get_lib().mopt_flat_init(d.data_ptr(), c.data_ptr(), len(chunks),
                                                 _lib.stream_ptr(self.device)), "flat_init")
        if fills is None:
            self.init_aux(slot)

    def update_hparams(self, slot: int, **changes) -> None:
        cfg = dataclasses.replace(self.members[slot], **changes)
        self.members[slot] = cfg
        self._write_hp(slot, cfg, int(self.hp[slot]["t"]))

    def remove_member(self, slot: int) -> None:
        self.members[slot] = None
        self.hp[slot]["t"] = 0
        self.opt_hp[slot] = 0

    def steps_done(self, slot: int) -> int:
        return int(self.hp[slot]["t"])

    # ------------------------------------------------------------------ training
    def _expand(self, t: torch.Tensor, dtype=None) -> torch.Tensor:
        """The shared batch of every trial, with a leading population dimension."""
        t = t.to(self.device) if dtype is None else t.to(self.device, dtype)
        return t.unsqueeze(0).expand(self.capacity, *t.shape).contiguous()

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """One optimizer step of every member on the shared batch (x, y).

        On a GPU the whole step -- forward, backward, gradient clipping and the fused optimizer
        -- is captured once into a HIP graph and replayed (the per-step host cost of autograd
        and ~100 launches is what bounds small models such as ResNet-20); the per-trial
        hyper-parameters and step counters reach the graph through a static device buffer.
        """
        active = np.array([m is not None for m in self.members])
        self.hp["t"][active] += 1
        self.opt_hp["t"] = self.hp["t"]
        from ..ops import _lib
        # under MOPT_SYNC_CHECK / MOPT_KERNEL_CHECKED every launch is checked eagerly
        if self.use_graph and self.device.type == "cuda" and not _lib.SYNC_CHECK:
            self._graph_step(x, y)
            return
        self._body(x, y, None)

    def _body(self, x, y, hp_dev):
        for a, b in self._zero_runs:
            self.g16[a:b].zero_()
        out = self._loss(x, y, train=True)
        loss = out[0] if isinstance(out, tuple) else out
        # d(sum loss) / d loss_p = 1: a persistent ones vector (created in the eager warm-up
        # before any graph capture) instead of loss.sum() -- no reduction and no fill per step
        ones = getattr(self, "_loss_ones", None)
        if ones is None or ones.shape != loss.shape or ones.device != loss.device:
            ones = self._loss_ones = torch.ones_like(loss)
        loss.backward(ones)
        P = self.capacity
        self.stats[:P].copy_(loss.detach())
        if isinstance(out, tuple):
            self.stats[P:2 * P].copy_(out[1].detach())
        with torch.no_grad():
            self.opt.step(self.master_buf, self.p16, self.g16, self.m, self.v, self.opt_hp,
                          hp_dev=hp_dev)

    def _graph_step(self, x, y):
        from ..ops._lib import upload_bytes_into
        if self._graph is None or self._gx.shape != x.shape or self._gy.shape != y.shape:
            self._capture(x, y)
        self._gx.copy_(x)
        self._gy.copy_(y)
        upload_bytes_into(self._hp_dev, self.opt_hp)
        self._graph.replay()

    def _capture(self, x, y):
        from ..ops._lib import upload_bytes
        self._gx = x.detach().clone()
        self._gy = y.detach().clone()
        self._hp_dev = upload_bytes(self.opt_hp, self.device)
        state = [self.master_buf, self.p16, self.m, self.v, self.aux, self.stats]
        backup = [t.clone() for t in state]
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):          # warm-up: library handles, allocator pools, autograd
                self._body(self._gx, self._gy, self._hp_dev)
        torch.cuda.current_stream(self.device).wait_stream(side)
        with torch.no_grad():
            for t, b in zip(state, backup):
                t.copy_(b)
        del backup
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self._body(self._gx, self._gy, self._hp_dev)
        self._graph = graph

    # ------------------------------------------------------------------ evaluation / stats
    @torch.no_grad()
    def evaluate_async(self, x, y, slots=None):
        out = self._loss(x, y, train=False)
        P = self.capacity
        loss = out[0] if isinstance(out, tuple) else out
        self.stats[2 * P:3 * P].copy_(loss)
        if isinstance(out, tuple):
            self.stats[3 * P:].copy_(out[1])
        return {"rows": self.rows_per_batch(x), "subset": None if slots is None
                else set(int(s) for s in slots)}

    def device_busy(self):
        return device_busy(self.device)

    def stats_snapshot(self) -> np.ndarray:
        return self.stats.cpu().numpy().reshape(4, self.capacity)

    def train_rows(self) -> int:
        return self.batch_size

    def stats_snapshot_async(self):
        from ..ops.population import StatsSnapshot
        return StatsSnapshot(self.stats, self.capacity)

    def raw_results(self, snap, handle, rows=None):
        """(train loss, eval loss, eval secondary) per slot from a snapshot, unmasked."""
        tl = snap[0].astype(np.float64) / self.train_rows()
        if handle is None:
            nan = np.full(self.capacity, np.nan)
            return tl, nan, nan
        rows = handle["rows"]
        loss = snap[2].astype(np.float64) / rows
        second = (np.exp(np.minimum(loss, 50.0)) if self.secondary == "ppl"
                  else snap[3].astype(np.float64) / rows)
        return tl, loss, second

    def train_loss(self, snap=None) -> np.ndarray:
        snap = self.stats_snapshot() if snap is None else snap
        out = snap[0].astype(np.float64) / self.train_rows()
        out[[m is None for m in self.members]] = np.nan
        return out

    def eval_result(self, snap, handle):
        rows = handle["rows"]
        loss = snap[2].astype(np.float64) / rows
        second = (np.exp(np.minimum(loss, 50.0)) if self.secondary == "ppl"
                  else snap[3].astype(np.float64) / rows)
        for s in range(self.capacity):
            if self.members[s] is None or (handle["subset"] is not None
                                           and s not in handle["subset"]):
                loss[s] = second[s] = np.nan
        return loss, second

    def evaluate(self, x, y, slots=None):
        handle = self.evaluate_async(x, y, slots)    # before the snapshot that reads its sums
        return self.eval_result(self.stats_snapshot(), handle)

    # ------------------------------------------------------------------ checkpoints
    @property
    def master_buf(self) -> torch.Tensor:
        """The master weights' own buffer: f32, or the int16 low halves of the split master."""
        return self.plo if self.split else self.p32

    def _master_slice(self, sl) -> torch.Tensor:
        """f32 master weights of flat range ``sl`` (a copy when split)."""
        if self.split:
            from ..ops.reference import join_f32
            return join_f32(self.p16[sl], self.plo[sl])
        return self.p32[sl]

    def _set_master_slice(self, sl, values: torch.Tensor) -> None:
        """Master weights (and the bf16 working copy) of flat range ``sl`` from f32 values."""
        if self.split:
            from ..ops.reference import split_f32
            hi, lo = split_f32(values.to(self.device, torch.float32))
            self.p16[sl] = hi
            self.plo[sl] = lo
        else:
            self.p32[sl] = values
            self.p16[sl] = self.p32[sl].to(torch.bfloat16)

    def master_flat(self) -> torch.Tensor:
        """Every master weight as one f32 tensor (a copy when split; tests and tools)."""
        return self._master_slice(slice(0, self.n_flat))

    @torch.no_grad()
    def load_master_flat(self, values: torch.Tensor) -> None:
        """Set every master weight (and the working copy) from an f32 tensor."""
        self._set_master_slice(slice(0, self.n_flat), values)

    def _state_bufs(self):
        return [self.master_buf, self.m] + ([self.v] if self.v.numel() else [])

    def used_params_for(self, width=None) -> int:
        return self.n_params

    def alloc_ckpt_pool(self, n: int) -> None:
        k = len(self._state_bufs())
        self._ck = torch.zeros(n, k, self.n_params, dtype=torch.float32, device=self.device)
        self._ck_aux = torch.zeros(n, max(self.n_aux, 4), dtype=torch.float32, device=self.device)

    def _copy_items(self, slot, idx, to_pool: bool):
        from ..ops.ckpt import Split
        items = []
        for j, buf in enumerate(self._state_bufs()):
            o = 0
            for sl in self._slices(slot):
                n = sl.stop - sl.start
                pool = self._ck[idx, j, o:o + n]
                if j == 0 and self.split:        # the pool holds the joined f32 master
                    part = Split(self.p16[sl], self.plo[sl])
                    items.append((part, pool, None) if to_pool else (pool, None, part))
                elif to_pool:                    # (a bf16 moment widens to the f32 pool)
                    items.append((buf[sl], pool, None))
                elif buf.dtype == torch.bfloat16:   # ... and narrows back on load
                    items.append((pool, None, buf[sl]))
                else:
                    items.append((pool, buf[sl], self.p16[sl] if j == 0 else None))
                o += n
        o = 0
        for x in self._aux_slices(slot):
            n = x.stop - x.start
            pool = self._ck_aux[idx, o:o + n]
            items.append((self.aux[x], pool, None) if to_pool else (pool, self.aux[x], None))
            o += n
        return items

    @torch.no_grad()
    def save_states(self, pairs) -> list:
        from ..ops.ckpt import multi_copy
        items, metas = [], []
        for slot, idx in pairs:
            items += self._copy_items(slot, idx, True)
            metas.append({"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
                          "ck": int(idx), "n": self.n_params})
        multi_copy(items)
        return metas

    @torch.no_grad()
    def load_states(self, pairs) -> None:
        from ..ops.ckpt import multi_copy
        items = []
        for slot, meta in pairs:
            items += self._copy_items(slot, meta["ck"], False)
            cfg = MemberConfig(**meta["config"])
            self.members[slot] = cfg
            self._write_hp(slot, cfg, int(meta["t"]))
        multi_copy(items)

    def pool_state(self, meta: dict) -> dict:
        idx = meta["ck"]
        st = {"config": meta["config"], "t": meta["t"], "p32": self._ck[idx, 0],
              "m32": self._ck[idx, 1], "aux": self._ck_aux[idx, :self.n_aux],
              "optimizer": self.optimizer}
        if self.v.numel():
            st["v32"] = self._ck[idx, 2]
        return st

    def slot_state(self, slot: int) -> dict:
        cat = lambda buf: torch.cat([buf[sl] for sl in self._slices(slot)])  # noqa: E731
        st = {"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
              "p32": torch.cat([self._master_slice(sl) for sl in self._slices(slot)]),
              "m32": cat(self.m).float(), "aux": self._aux_of(slot),
              "optimizer": self.optimizer}
        if self.v.numel():
            st["v32"] = cat(self.v)
        return st

    @torch.no_grad()
    def load_slot_state(self, slot: int, state: dict) -> None:
        o = 0
        for sl in self._slices(slot):
            n = sl.stop - sl.start
            self._set_master_slice(sl, state["p32"][o:o + n])
            self.m[sl] = state["m32"][o:o + n]
            if self.v.numel():
                self.v[sl] = state["v32"][o:o + n]
            o += n
        if "aux" in state and self.n_aux:
            self._set_aux(slot, state["aux"])
        cfg = MemberConfig(**state["config"])
        self.members[slot] = cfg
        self._write_hp(slot, cfg, int(state["t"]))

    @torch.no_grad()
    def copy_member(self, src: int, dst: int, **hp_changes) -> None:
        """PBT exploit inside one device: dst <- src (weights, optimizer state, step count)."""
        for a, b in zip(self._slices(src), self._slices(dst)):
            for buf in [self.p16] + self._state_bufs():
                buf[b] = buf[a]
        for a, b in zip(self._aux_slices(src), self._aux_slices(dst)):
            self.aux[b] = self.aux[a]
        cfg = dataclasses.replace(self.members[src], **hp_changes)
        self.members[dst] = cfg
        self._write_hp(dst, cfg, int(self.hp[src]["t"]))

    # ---- C4 straight from / into the checkpoint pool (PopulationSweep._exchange_checkpoints)
    def _c4_header(self) -> torch.Tensor:
        return torch.empty(2 + self.n_aux, dtype=torch.float32, device=self.device)

    def c4_send_tensors(self, meta: dict) -> list:
        """The pool entry of a checkpoint as it stands ([state buffers, n_params] f32,
        contiguous) and a small header: step count, seed, the auxiliary state."""
        idx = meta["ck"]
        hdr = self._c4_header()
        head = torch.tensor([int(meta["t"]), int(meta["config"]["seed"])], dtype=torch.int32)
        hdr[:2].copy_(head.view(torch.float32))
        if self.n_aux:
            hdr[2:].copy_(self._ck_aux[idx, :self.n_aux])
        return [self._ck[idx], hdr]

    def c4_recv_tensors(self, idx: int) -> list:
        return [self._ck[idx], self._c4_header()]

    def c4_finish(self, idx: int, tensors: list) -> dict:
        """Pool meta of a checkpoint received into entry ``idx`` (for :meth:`load_states`)."""
        hdr = tensors[1]
        t, seed = (int(v) for v in hdr[:2].view(torch.int32).cpu().tolist())
        if self.n_aux:
            self._ck_aux[idx, :self.n_aux].copy_(hdr[2:])
        return {"config": MemberConfig(width=0, lr=0.0, seed=seed).to_dict(), "t": t,
                "ck": int(idx), "n": self.n_params}

    def _n_packed(self) -> int:
        return 2 + len(self._state_bufs()) * self.n_params + self.n_aux

    def empty_packed_state(self, width=None) -> torch.Tensor:
        return torch.empty(self._n_packed(), dtype=torch.float32, device=self.device)

    def pack_state(self, state: dict) -> torch.Tensor:
        head = torch.tensor([int(state["t"]), int(state["config"]["seed"])], dtype=torch.int32)
        parts = [head.view(torch.float32).to(self.device), state["p32"].reshape(-1),
                 state["m32"].reshape(-1)]
        if self.v.numel():
            parts.append(state["v32"].reshape(-1))
        aux = state.get("aux")
        parts.append(aux.reshape(-1) if aux is not None
                     else torch.zeros(self.n_aux, device=self.device))
        return torch.cat([p.to(self.device, torch.float32) for p in parts])

    def unpack_state(self, buf: torch.Tensor, width=None) -> dict:
        n = self.n_params
        t, seed = (int(v) for v in buf[:2].view(torch.int32).cpu().tolist())
        st = {"config": MemberConfig(width=0, lr=0.0, seed=seed).to_dict(), "t": t,
              "p32": buf[2:2 + n], "m32": buf[2 + n:2 + 2 * n], "optimizer": self.optimizer}
        o = 2 + 2 * n
        if self.v.numel():
            st["v32"] = buf[o:o + n]
            o += n
        st["aux"] = buf[o:]
        return st
