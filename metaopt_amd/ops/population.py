"""Device-resident population of MLP trials trained side by side (north-star configs 1 and 2).

:class:`PopulationMLP` owns flat device buffers for ``capacity`` trial *slots*:

* master weights: on the HIP backend ``p16`` (the bf16 working copy the forward reads) plus
  ``plo``, a 16-bit residual that makes (``p16``, ``plo``) an exact f32 master in 4 bytes
  (``csrc/common.h``); on the reference backend a plain f32 ``p32`` and its ``p16`` copy;
  ``m32``/``v32`` optimizer state -- every slot a fixed-size region sized for ``max_width``
  (288 GB of HBM makes the
  per-slot worst case cheap, and fixed regions make slot replacement, ASHA resume and PBT exploit
  plain region copies);
* ``act``/``grad`` bf16 activations and their gradients ([rows][N_l] per slot and layer);
* a hyper-parameter table (per-slot lr / momentum / weight decay / dropout / seed / step).

A trial with hidden width ``w`` uses padded dims (multiples of 64) inside its region; padding is
zero and stays zero (a zero-padded unit never receives gradient), so ragged widths cost only their
own padded FLOPs.  Each layer is one launch over a work list of (trial-layer, tile) items: the
forward (K1, K7), fused softmax-CE (K4) and the fused backward + SGD/AdamW update (K2, K5, K6)
kernels of ``csrc/pop_mlp.hip``.  Inside an interval (``train_steps``) the first layer's
backward + update of step t and its forward of step t + 1 run as one kernel
(``mlp_bwd0_fwd_kernel``: one pass over the largest weight matrix instead of two).

Backends: ``"hip"`` (gfx950 kernels, the only GPU path; never falls back silently) and
``"torch"`` (the fp32 reference of :mod:`metaopt_amd.ops.reference`, used on CPU-only hosts).
"""
from __future__ import annotations

import ctypes
import dataclasses
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from . import reference as ref

TL_DTYPE = np.dtype([("K", "<i4"), ("N", "<i4"), ("trial", "<i4"), ("n_real", "<i4"),
                     ("w_off", "<i8"), ("b_off", "<i8"), ("x_off", "<i8"), ("y_off", "<i8"),
                     ("gx_off", "<i8"), ("rows", "<i4"), ("k_real", "<i4")])
HP_DTYPE = np.dtype([("lr", "<f4"), ("b1", "<f4"), ("wd", "<f4"), ("drop", "<f4"),
                     ("b2", "<f4"), ("eps", "<f4"), ("seed", "<u4"), ("t", "<u4")])
INIT_DTYPE = np.dtype([("w_off", "<i8"), ("b_off", "<i8"), ("K", "<i4"), ("N", "<i4"),
                       ("k_real", "<i4"), ("n_real", "<i4"), ("seed", "<u4"), ("layer", "<i4"),
                       ("bound", "<f4"), ("pad", "<i4")])
assert TL_DTYPE.itemsize == 64 and HP_DTYPE.itemsize == 32 and INIT_DTYPE.itemsize == 48

TILE = 64
FWD_TN = 64             # hidden-layer forward tile width (csrc/pop_mlp.hip mopt_mlp_fwd)
MAX_ROWS = 64 * 128     # csrc/pop_mlp.hip mopt_mlp_bwd: at most 64 row blocks per launch
FWD_RELU, FWD_DROPOUT, FWD_WRITE_GRAD, FWD_STORE_STATS, FWD_COUNT_STEP = 1, 2, 4, 8, 16
FWD_NARROW_CE = 32      # loss layer with <= NARROW_CLASSES classes: 16 of its 64 W rows live
BWD_HAS_DX, BWD_IN_DROPOUT, BWD_UPDATE_BIAS, BWD_NARROW = 1, 2, 4, 8
NARROW_CLASSES = 16


class _MlpStep(ctypes.Structure):
    """Argument block of ``mopt_mlp_step`` (csrc/pop_mlp.hip ``MlpStep``): one host call
    launches a group's whole train step; built once per work-table refresh."""
    _fields_ = [("tls", ctypes.c_void_p), ("fwd", ctypes.c_void_p * 8),
                ("bwd", ctypes.c_void_p * 8), ("n_fwd", ctypes.c_int32 * 8),
                ("n_bwd", ctypes.c_int32 * 8), ("L", ctypes.c_int32), ("rb", ctypes.c_int32),
                ("drop", ctypes.c_int32), ("opt", ctypes.c_int32)] + \
               [(n, ctypes.c_void_p) for n in ("plo", "p16", "m32", "v32", "act", "grad", "hp",
                                               "loss", "correct")] + \
               [("inv_b", ctypes.c_float), ("n_stats", ctypes.c_int32),
                ("fwd_tn", ctypes.c_int32), ("narrow", ctypes.c_int32),
                ("bwd0f", ctypes.c_void_p), ("n_bwd0f", ctypes.c_int32),
                ("fuse0", ctypes.c_int32)]
OPTIMIZERS = {"sgd": 0, "adamw": 1}


def pad64(n: int) -> int:
    return (int(n) + TILE - 1) // TILE * TILE


def _ranges(counts: np.ndarray) -> np.ndarray:
    """concatenate(arange(c) for c in counts), vectorised."""
    counts = np.asarray(counts, dtype=np.int64)
    total = int(counts.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    starts = np.repeat(np.cumsum(counts) - counts, counts)
    return np.arange(total, dtype=np.int64) - starts


@dataclass
class MemberConfig:
    """Hyper-parameters of one population member (one trial)."""

    width: int
    lr: float
    momentum: float = 0.9          # SGD momentum, or AdamW beta1
    weight_decay: float = 0.0
    dropout: float = 0.0
    seed: int = 0
    beta2: float = 0.999
    eps: float = 1e-8
    batch_size: int = 0            # rows per step (a multiple of 128); 0 = the population's batch

    def to_dict(self) -> dict:
        # field by field (dataclasses.asdict deep-copies recursively: a visible cost when the
        # sweep checkpoints a hundred members per sync)
        return {f: getattr(self, f) for f in _MEMBER_FIELDS}


_MEMBER_FIELDS = tuple(f.name for f in dataclasses.fields(MemberConfig))


class StatsSnapshot:
    """Device->host copy of a population's ``[4, capacity]`` statistics queued on the current
    stream (pinned, non-blocking): :meth:`get` waits for that copy only, so the host can read
    the statistics of an earlier sync while the GPU already trains the next interval."""

    __slots__ = ("capacity", "rows", "_host", "_ev")

    def __init__(self, stats: torch.Tensor, capacity: int, rows=None):
        self.capacity = capacity
        self.rows = rows          # per-slot train rows when the copy was queued (or None)
        if stats.device.type == "cuda":
            self._host = torch.empty(stats.shape, dtype=stats.dtype, pin_memory=True)
            self._host.copy_(stats, non_blocking=True)
            self._ev = torch.cuda.Event()
            self._ev.record(torch.cuda.current_stream(stats.device))
        else:
            self._host = stats.detach().clone()
            self._ev = None

    def ready(self) -> bool:
        return self._ev is None or self._ev.query()

    def get(self) -> np.ndarray:
        if self._ev is not None:
            self._ev.synchronize()
            self._ev = None
        return self._host.numpy().reshape(4, self.capacity)


N_XCD = 8


def _xcd_schedule(trial: np.ndarray, cost: np.ndarray, n_xcd: int = N_XCD) -> np.ndarray:
    """Work-list permutation that balances the launch over the XCDs.

    The MLP kernels run work item ``blockIdx.x`` (csrc/pop_mlp.hip), and workgroups are dealt to
    the XCDs round-robin (blocks b and b + 8 share one: speed only, never correctness), so
    position ``8 i + x`` of the list is the ``i``-th item of XCD ``x``.  Items (given grouped by
    trial) are assigned to XCDs by total cost, longest first: a whole trial to the least-loaded
    XCD (its tiles share its operands in that XCD's L2), a trial heavier than half an XCD's share
    in contiguous pieces of about a quarter share.  Each XCD's items then run longest first, and
    the shorter XCD lists are padded with ``-1`` (a no-op workgroup).  The previous scheme, equal
    item COUNTS per XCD, left one XCD with up to 1.5x the work of another (bwd0: the slowest
    XCD at 122 % of the mean, scripts/dev/sched_sim.py).  Returns indices into the items, -1 =
    padding."""
    n = len(cost)
    if n == 0:
        return np.zeros(0, np.int64)
    cost = np.asarray(cost, dtype=np.float64)
    bounds = np.flatnonzero(np.r_[True, trial[1:] != trial[:-1], True])
    groups = [(int(bounds[g]), int(bounds[g + 1])) for g in range(len(bounds) - 1)]
    csum = np.r_[0.0, np.cumsum(cost)]
    share = csum[-1] / n_xcd
    pieces = []                      # (cost, start, stop)
    for a, b in groups:
        c = csum[b] - csum[a]
        if c <= share / 2 or b - a == 1:
            pieces.append((c, a, b))
            continue
        k = max(2, int(np.ceil(c / (share / 4))))
        cuts = np.searchsorted(csum[a:b + 1] - csum[a], np.linspace(0, c, k + 1)[1:-1])
        edges = [a] + sorted({a + int(x) for x in cuts if 0 < x < b - a}) + [b]
        pieces += [(csum[e1] - csum[e0], e0, e1) for e0, e1 in zip(edges[:-1], edges[1:])]
    pieces.sort(key=lambda t: (-t[0], t[1]))
    load = np.zeros(n_xcd)
    lists = [[] for _ in range(n_xcd)]
    for c, a, b in pieces:
        x = int(np.argmin(load))
        load[x] += c
        lists[x].extend(range(a, b))
    width = max(len(l) for l in lists)
    out = np.full((width, n_xcd), -1, dtype=np.int64)
    for x, l in enumerate(lists):
        if l:
            idx = np.asarray(l, dtype=np.int64)
            out[:len(l), x] = idx[np.argsort(-cost[idx], kind="stable")]
    return out.reshape(-1)


def _reschedule(w: np.ndarray, group_of: np.ndarray, g: int, L: int, tl: np.ndarray,
                field: str) -> np.ndarray:
    """The real items of work list ``w`` whose slot is in group ``g`` (``group_of[slot]``),
    rescheduled over the XCDs (a trial's items kept in their order)."""
    w = w[w[:, 0] >= 0]
    w = w[group_of[w[:, 0] // L] == g]
    w = w[np.lexsort((w[:, 1], w[:, 0]))]
    return _work_list(w[:, 0], w[:, 1], tl[field][w[:, 0]])


def _work_list(tl_index: np.ndarray, tile: np.ndarray, cost: np.ndarray) -> np.ndarray:
    """[n, 2] int32 work list (trial-layer, tile) in :func:`_xcd_schedule` order; padding
    entries are (-1, 0)."""
    order = _xcd_schedule(tl_index, cost)
    w = np.zeros((len(order), 2), np.int32)
    w[:, 0] = -1
    real = order >= 0
    w[real, 0] = tl_index[order[real]]
    w[real, 1] = tile[order[real]]
    return w


def _lib_sync_check() -> bool:
    from . import _lib
    return _lib.SYNC_CHECK


class _SplitBuffer:
    """(hi, lo) split-master buffers sliced together (``buf[a:b]`` -> ckpt.Split)."""

    def __init__(self, hi, lo):
        self.hi, self.lo = hi, lo

    def __getitem__(self, sl):
        from .ckpt import Split
        return Split(self.hi[sl], self.lo[sl])


def device_busy(device):
    if torch.device(device).type != "cuda":
        return lambda: True
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    return lambda: not ev.query()


class PopulationMLP:
    """``capacity`` MLP trials (``n_hidden`` ReLU layers of per-trial width) on one device."""

    def __init__(self, capacity: int, in_features: int = 784, num_classes: int = 10,
                 max_width: int = 1024, n_hidden: int = 3, batch_size: int = 128,
                 eval_batch: int = 1024, optimizer: str = "sgd", device=None,
                 backend: Optional[str] = None, emulate_bf16: bool = True,
                 n_streams: Optional[int] = None, momentum_dtype: str = "fp32"):
        if optimizer not in OPTIMIZERS:
            raise ValueError(f"optimizer must be one of {sorted(OPTIMIZERS)}")
        if momentum_dtype not in ("fp32", "bf16"):
            raise ValueError("momentum_dtype must be 'fp32' or 'bf16'")
        if momentum_dtype == "bf16" and optimizer != "sgd":
            raise ValueError("the bf16 momentum buffer is an SGD option")
        if num_classes > TILE:
            raise ValueError("the fused CE epilogue supports at most 64 classes")
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        if backend is None:
            backend = "hip" if self.device.type == "cuda" else "torch"
        if backend == "hip":
            if self.device.type != "cuda":
                raise ValueError("the hip backend needs a GPU device")
            from . import _lib
            self._lib = _lib.get_lib()  # raises loudly: no silent fallback on a GPU box
        # HIP weight layout: k-strip-major [K/64][N][64] (csrc/pop_mlp.hip w_row_stride) -- the
        # optimizer state shares it; layer_views() returns row-major copies
        self.w_strip = backend == "hip" and self._lib.mopt_mlp_w_layout() == 1
        # output features per hidden-layer forward work item (csrc/pop_mlp.hip mlp_fwd_kernel TN)
        self.fwd_tn = FWD_TN
        self.backend = backend
        # the population's trials are split into ``n_streams`` groups of equal cost whose train
        # steps run on their own HIP streams, unsynchronised between syncs: one group's
        # latency-bound forward overlaps another's bandwidth-bound backward (measured: two
        # processes sharing the GPU ran 14% more trials/s than one).  Any other operation first
        # joins the side streams into the main one (``_join``); the next train step forks them
        # again after it.  Default 3 (round 5, one box, headline bench, two repetitions each:
        # 1 / 3 / 4 / 6 / 8 streams = 786-790 / 827-831 / 826-827 / 722-737 / 720-724 trials/s --
        # in situ the forward kernels run at ~2.3 TB/s against ~4.8 for the backward, and the
        # other groups' kernels fill those latency-bound phases and every kernel's tail; past
        # the process's 4 hardware queues (GPU_MAX_HW_QUEUES) streams share queues and lose;
        # profiles/round5.md).  Round 3, before the one-call interval launch, measured 1 vs 2
        # streams as noise.
        if n_streams is None:
            n_streams = int(os.environ.get("MOPT_STREAMS", "3")) if backend == "hip" else 1
        self.n_streams = max(1, int(n_streams))
        # consecutive train steps of one interval fuse the first layer's backward + update with
        # the next step's first-layer forward (csrc/pop_mlp.hip mlp_bwd0_fwd_kernel: one pass
        # over W0 instead of two; bit-identical results).  MOPT_FUSE0=0 keeps the separate
        # launches (the A/B and the equality test).
        self.fuse_first_layer = os.environ.get("MOPT_FUSE0", "1") != "0"
        # train_steps queues the groups' steps round-robin, this many at a time (0: each group's
        # whole interval in turn -- the groups then start and finish one after the other)
        self.step_chunk = int(os.environ.get("MOPT_STEP_CHUNK", "4"))
        self._side_streams: list = []
        self._events: list = []
        self._parts: list = []
        self._side_pending = False    # side streams hold work the main stream has not joined
        self._fork_needed = True      # the main stream holds work the side streams must follow
        if batch_size % 128 or eval_batch % 128 or batch_size < 128:
            raise ValueError("batch sizes must be multiples of 128")
        if batch_size > MAX_ROWS:
            raise ValueError(f"batch_size above {MAX_ROWS} (64 row blocks of 128)")
        self.capacity = int(capacity)
        self.in_features = int(in_features)
        self.num_classes = int(num_classes)
        self.max_width = int(max_width)
        self.n_hidden = int(n_hidden)
        self.L = self.n_hidden + 1
        self.batch_size = int(batch_size)
        self.eval_batch = int(eval_batch)
        self.optimizer = optimizer
        # SGD momentum kept in bf16 (RNE after each update, the rounded value drives the weight
        # update): 14 instead of 18 bytes per parameter and step through the fused backward
        self.momentum_dtype = momentum_dtype
        self.emulate_bf16 = emulate_bf16
        self.K0 = pad64(in_features)

        dims_max = self.layer_dims(self.max_width)
        self.slot_params = sum(pad64(k * n) + pad64(n) for k, n in dims_max)
        self.nmax = [n for _, n in dims_max]
        self.act_row = sum(self.nmax)
        dev = self.device
        total = self.capacity * self.slot_params
        # HIP: split master (hi = p16, lo = plo; no separate f32 copy to write every step)
        self.split = backend == "hip"
        self.p32 = None if self.split else torch.zeros(total, dtype=torch.float32, device=dev)
        self.plo = torch.zeros(total, dtype=torch.int16, device=dev) if self.split else None
        self.p16 = torch.zeros(total, dtype=torch.bfloat16, device=dev)
        self.m32 = torch.zeros(total, dtype=torch.bfloat16 if momentum_dtype == "bf16"
                               else torch.float32, device=dev)   # momentum / AdamW first moment
        self.v32 = (torch.zeros(total, dtype=torch.float32, device=dev) if optimizer == "adamw"
                    else torch.zeros(1, dtype=torch.float32, device=dev))
        self.act = torch.zeros(self.capacity * self.batch_size * self.act_row,
                               dtype=torch.bfloat16, device=dev)
        self.grad = torch.zeros_like(self.act)
        self.act_eval = torch.zeros(self.capacity * self.eval_batch * self.act_row,
                                    dtype=torch.bfloat16, device=dev)
        # per-slot loss sum and #correct of the last train step and of the last evaluation, in
        # one buffer: one zeroing launch per step, one device->host copy per sync
        P = self.capacity
        self.stats = torch.zeros(4 * P, dtype=torch.float32, device=dev)
        self.loss, self.correct = self.stats[:P], self.stats[P:2 * P]
        self.eval_loss, self.eval_correct = self.stats[2 * P:3 * P], self.stats[3 * P:]
        self.hp = np.zeros(self.capacity, dtype=HP_DTYPE)
        self.hp_dev = torch.zeros(self.capacity * HP_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        self.members: List[Optional[MemberConfig]] = [None] * self.capacity
        self._rows_np = np.full(self.capacity, self.batch_size, dtype=np.float64)
        self._pending_init = set()
        self._dirty = True
        self._tables: Dict[str, dict] = {}

    # ------------------------------------------------------------------ layout
    def layer_dims(self, width: int):
        """Padded (K, N) per layer for a trial of hidden width ``width``."""
        wp = pad64(width)
        if self.n_hidden == 0:
            return [(self.K0, TILE)]
        dims = [(self.K0, wp)]
        dims += [(wp, wp)] * (self.n_hidden - 1)
        dims.append((wp, TILE))
        return dims

    def real_dims(self, width: int):
        if self.n_hidden == 0:
            return [(self.in_features, self.num_classes)]
        dims = [(self.in_features, width)]
        dims += [(width, width)] * (self.n_hidden - 1)
        dims.append((width, self.num_classes))
        return dims

    def param_offsets(self, width: int):
        """[(w_off, b_off)] per layer, relative to the slot base."""
        offs, o = [], 0
        for k, n in self.layer_dims(width):
            offs.append((o, o + pad64(k * n)))
            o += pad64(k * n) + pad64(n)
        return offs

    def slot_base(self, slot: int) -> int:
        return slot * self.slot_params

    def n_params(self, slot: int) -> int:
        """Real (unpadded) parameter count of the member in ``slot``."""
        cfg = self.members[slot]
        return sum(k * n + n for k, n in self.real_dims(cfg.width))

    def padded_params(self, slot: int) -> int:
        cfg = self.members[slot]
        return sum(k * n + n for k, n in self.layer_dims(cfg.width))

    def flops_per_step(self, slot: int) -> int:
        """Padded MFMA FLOPs of one train step (fwd + dX + dW) of the member in ``slot``."""
        cfg = self.members[slot]
        f, rows = 0, self.member_rows(cfg)
        for l, (k, n) in enumerate(self.layer_dims(cfg.width)):
            f += 2 * rows * k * n * (3 if l > 0 else 2)
        return f

    def bytes_per_step(self, slot: int) -> int:
        """HBM bytes per step for parameters/state of ``slot`` (fwd bf16 + fused bwd/update)."""
        w = 8 if self.split else 10      # split master r+w (4+4) vs f32 r+w + bf16 copy w
        per = 2 + w + (16 if self.optimizer == "adamw" else
                       4 if self.momentum_dtype == "bf16" else 8)
        return per * self.padded_params(slot)

    # ------------------------------------------------------------------ members
    def member_rows(self, cfg: MemberConfig) -> int:
        """Rows per train step of a member: its own batch size, or the population's.  A member
        with a smaller batch trains on the first rows of each (population-sized) minibatch; its
        loss and gradient are means over its own rows (TL ``rows``, csrc/pop_mlp.hip)."""
        return int(cfg.batch_size) or self.batch_size

    def _check_member(self, cfg: MemberConfig) -> None:
        if cfg.width > self.max_width or cfg.width < 1:
            raise ValueError(f"width {cfg.width} outside [1, {self.max_width}]")
        if not (0.0 <= cfg.dropout < 1.0):
            raise ValueError("dropout must be in [0, 1)")
        b = int(cfg.batch_size)
        if b and (b % 128 or b < 0 or b > self.batch_size):
            raise ValueError(f"member batch_size {b} must be a multiple of 128 and <= the "
                             f"population's {self.batch_size}")

    def active_slots(self) -> List[int]:
        return [i for i, m in enumerate(self.members) if m is not None]

    def free_slots(self) -> List[int]:
        return [i for i, m in enumerate(self.members) if m is None]

    def _write_hp(self, slot: int, cfg: MemberConfig, t: int) -> None:
        self.hp[slot] = (cfg.lr, cfg.momentum, cfg.weight_decay, cfg.dropout, cfg.beta2, cfg.eps,
                         cfg.seed & 0xFFFFFFFF, t)

    def _upload_hp(self) -> None:
        from ._lib import upload_bytes_into
        upload_bytes_into(self.hp_dev, self.hp)

    def set_member(self, slot: int, cfg: MemberConfig, init: bool = True) -> None:
        """Place ``cfg`` in ``slot``; with ``init`` draw fresh weights (torch.nn.Linear-style
        U(-1/sqrt(fan_in), 1/sqrt(fan_in)) from the member's counter-based RNG stream).

        Initialisation is deferred and batched: every member set before the next train/eval call
        is initialised by one kernel launch."""
        self._check_member(cfg)
        self.members[slot] = cfg
        self._write_hp(slot, cfg, 0)
        if init:
            self._pending_init.add(slot)
        self._dirty = True

    def update_hparams(self, slot: int, **changes) -> None:
        """Change hyper-parameters of a live member without touching its weights (PBT explore)."""
        cfg = dataclasses.replace(self.members[slot], **changes)
        if cfg.width != self.members[slot].width:
            raise ValueError("width cannot change in place")
        self._check_member(cfg)
        t = int(self.hp[slot]["t"])
        self.members[slot] = cfg
        self._write_hp(slot, cfg, t)
        self._dirty = True

    def remove_member(self, slot: int) -> None:
        self._pending_init.discard(slot)
        self.members[slot] = None
        self.hp[slot] = np.zeros((), dtype=HP_DTYPE)
        self._dirty = True

    def steps_done(self, slot: int) -> int:
        return int(self.hp[slot]["t"])

    def _region(self, slot: int):
        b = self.slot_base(slot)
        return slice(b, b + self.slot_params)

    def _init_descs(self, slots) -> np.ndarray:
        """One InitDesc per (member, layer), vectorised over the members."""
        slots = np.asarray(list(slots), dtype=np.int64)
        L = self.L
        out = np.zeros((len(slots), L), dtype=INIT_DTYPE)
        if not len(slots):
            return out.reshape(-1)
        widths = np.array([self.members[s].width for s in slots], dtype=np.int64)
        seeds = np.array([self.members[s].seed & 0xFFFFFFFF for s in slots], dtype=np.uint32)
        wp = (widths + TILE - 1) // TILE * TILE
        base = slots * self.slot_params
        off = np.zeros_like(base)
        for l in range(L):
            if self.n_hidden == 0:
                K, N = np.full_like(wp, self.K0), np.full_like(wp, TILE)
                kr, nr = np.full_like(wp, self.in_features), np.full_like(wp, self.num_classes)
            else:
                K = np.full_like(wp, self.K0) if l == 0 else wp
                N = np.full_like(wp, TILE) if l == L - 1 else wp
                kr = np.full_like(wp, self.in_features) if l == 0 else widths
                nr = np.full_like(wp, self.num_classes) if l == L - 1 else widths
            wsz = (K * N + TILE - 1) // TILE * TILE
            r = out[:, l]
            r["w_off"] = base + off
            r["b_off"] = base + off + wsz
            r["K"], r["N"], r["k_real"], r["n_real"] = K, N, kr, nr
            r["seed"], r["layer"] = seeds, l
            r["bound"] = (np.float32(1.0) / np.sqrt(kr.astype(np.float32))).astype(np.float32)
            off = off + wsz + (N + TILE - 1) // TILE * TILE
        return out.reshape(-1)

    def _run_pending_init(self) -> None:
        if not self._pending_init:
            return
        self._join()
        slots = sorted(s for s in self._pending_init if self.members[s] is not None)
        self._pending_init.clear()
        if not slots:
            return
        descs = self._init_descs(slots)
        if self.backend == "hip":
            from ._lib import check, stream_ptr
            from ._lib import upload_bytes
            d = upload_bytes(descs, self.device)
            check(self._lib.mopt_mlp_init(d.data_ptr(), len(descs), self.plo.data_ptr(),
                                          self.p16.data_ptr(), self.m32.data_ptr(),
                                          self.v32.data_ptr(),
                                          int(self.optimizer == "adamw")
                                          | (2 if self.momentum_dtype == "bf16" else 0),
                                          stream_ptr(self.device)), "mlp_init")
            self._init_keep = d  # keep the descriptor alive until the launch has run
        else:
            for row in descs:
                ref.init_layer(self.p32, self.m32, self.v32 if self.optimizer == "adamw" else None,
                               int(row["w_off"]), int(row["b_off"]), int(row["K"]), int(row["N"]),
                               int(row["k_real"]), int(row["n_real"]), int(row["seed"]),
                               int(row["layer"]), float(row["bound"]))
            for s in slots:
                b = self.slot_base(s)
                n = self.used_params(s)
                self.p16[b:b + n] = ref.split_f32(self.p32[b:b + n])[0]

    def layer_views(self, slot: int, buf: torch.Tensor = None):
        """[(W [N,K], b [N])] views of ``buf`` (default: f32 master) for the member in ``slot``
        (row-major copies of the weights when the HIP layout is k-strip-major)."""
        self._run_pending_init()
        self._join()
        cfg = self.members[slot]
        base = self.slot_base(slot)
        if buf is None and self.split:     # a decoded copy of the slot's f32 master
            buf, base = self.master(slot), 0
        buf = self.p32 if buf is None else buf
        out = []
        for (k, n), (wo, bo) in zip(self.layer_dims(cfg.width), self.param_offsets(cfg.width)):
            w = buf[base + wo: base + wo + n * k]
            w = (w.view(k // TILE, n, TILE).permute(1, 0, 2).reshape(n, k) if self.w_strip
                 else w.view(n, k))
            out.append((w, buf[base + bo: base + bo + n]))
        return out

    # ------------------------------------------------------------------ checkpoints (device)
    def master(self, slot: int) -> torch.Tensor:
        """The f32 master weights of ``slot``'s used region (a copy on the HIP backend)."""
        self._run_pending_init()
        self._join()
        b, n = self.slot_base(slot), self.used_params(slot)
        if self.split:
            return ref.join_f32(self.p16[b:b + n], self.plo[b:b + n])
        return self.p32[b:b + n]

    def _set_master(self, b: int, values: torch.Tensor) -> None:
        n = values.numel()
        values = values.to(self.device, torch.float32)
        if self.split:
            hi, lo = ref.split_f32(values)
            self.p16[b:b + n] = hi
            self.plo[b:b + n] = lo
        else:
            self.p32[b:b + n] = values
            self.p16[b:b + n] = ref.split_f32(values)[0]

    def used_params(self, slot: int) -> int:
        """Length of the prefix of the slot region the member actually uses."""
        return self.used_params_for(self.members[slot].width)

    def used_params_for(self, width: int) -> int:
        cache = self.__dict__.setdefault("_used_cache", {})
        n = cache.get(width)
        if n is None:
            n = cache[width] = sum(pad64(k * n) + pad64(n) for k, n in self.layer_dims(width))
        return n

    # -- checkpoint pool: batched save / restore of members (one kernel launch each) ------------
    def alloc_ckpt_pool(self, n: int) -> None:
        """``n`` checkpoint slots, each as large as a population slot (f32 master weights and
        optimizer state; 288 GB of HBM holds thousands)."""
        self.ck = torch.zeros(n, self._n_state_buffers(), self.slot_params, dtype=torch.float32,
                              device=self.device)

    def _state_tensors(self):
        w = _SplitBuffer(self.p16, self.plo) if self.split else self.p32
        return [w, self.m32] + ([self.v32] if self.optimizer == "adamw" else [])

    def _state_descs(self, slots, idxs, ns, save: bool) -> np.ndarray:
        """multi_copy descriptors between slot regions and checkpoint-pool entries, built with
        numpy from raw pointers (one row per member and state buffer)."""
        from .ckpt import DESC_DTYPE
        slots = np.asarray(slots, dtype=np.uint64)
        idxs = np.asarray(idxs, dtype=np.uint64)
        ns = np.asarray(ns, dtype=np.int64)
        SP = np.uint64(self.slot_params)
        nb = self._n_state_buffers()
        base = slots * SP
        ck0 = np.uint64(self.ck.data_ptr()) + np.uint64(4) * idxs * np.uint64(nb) * SP
        out = np.zeros((nb, len(slots)), dtype=DESC_DTYPE)
        out["n"] = ns
        m16 = self.m32.dtype == torch.bfloat16
        p16, plo = np.uint64(self.p16.data_ptr()), np.uint64(self.plo.data_ptr())
        m_ptr, v_ptr = np.uint64(self.m32.data_ptr()), np.uint64(self.v32.data_ptr())
        two, four = np.uint64(2), np.uint64(4)
        for j in range(nb):
            ckj = ck0 + four * np.uint64(j) * SP
            r = out[j]
            if save:
                r["dst"] = ckj
                if j == 0:
                    r["src16"], r["src_lo"] = p16 + two * base, plo + two * base
                elif j == 1 and m16:
                    r["src16"] = m_ptr + two * base
                else:
                    r["src"] = (m_ptr if j == 1 else v_ptr) + four * base
            else:
                r["src"] = ckj
                if j == 0:
                    r["dst16"], r["dst_lo"] = p16 + two * base, plo + two * base
                elif j == 1 and m16:
                    r["dst16"] = m_ptr + two * base
                else:
                    r["dst"] = (m_ptr if j == 1 else v_ptr) + four * base
        return out.reshape(-1)

    def save_states(self, pairs) -> list:
        """Checkpoint members: ``pairs`` = [(slot, pool index)]; returns per-member metadata."""
        from .ckpt import launch_descs, multi_copy
        self._run_pending_init()
        self._join()
        if self.split and self.device.type == "cuda":
            ns = [self.used_params(s) for s, _ in pairs]
            launch_descs(self._state_descs([s for s, _ in pairs], [i for _, i in pairs], ns,
                                           save=True), self.device)
            return [{"config": self.members[s].to_dict(), "t": int(self.hp[s]["t"]),
                     "ck": int(i), "n": n} for (s, i), n in zip(pairs, ns)]
        items, metas = [], []
        for slot, idx in pairs:
            n = self.used_params(slot)
            b = self.slot_base(slot)
            for j, buf in enumerate(self._state_tensors()):
                items.append((buf[b:b + n], self.ck[idx, j, :n], None))
            metas.append({"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
                          "ck": int(idx), "n": n})
        multi_copy(items)
        return metas

    def load_states(self, pairs) -> None:
        """Restore members from the pool: ``pairs`` = [(slot, metadata)] (bf16 copy included)."""
        from .ckpt import launch_descs, multi_copy
        self._join()
        if self.split and self.device.type == "cuda":
            launch_descs(self._state_descs([s for s, _ in pairs], [m["ck"] for _, m in pairs],
                                           [m["n"] for _, m in pairs], save=False), self.device)
            for slot, meta in pairs:
                self._pending_init.discard(slot)
                cfg = MemberConfig(**meta["config"])
                self.members[slot] = cfg
                self._write_hp(slot, cfg, int(meta["t"]))
            self._dirty = True
            return
        items = []
        for slot, meta in pairs:
            n, idx = meta["n"], meta["ck"]
            b = self.slot_base(slot)
            for j, buf in enumerate(self._state_tensors()):
                if isinstance(buf, _SplitBuffer):  # f32 pool -> split master (hi, lo)
                    items.append((self.ck[idx, j, :n], None, buf[b:b + n]))
                elif buf.dtype == torch.bfloat16:   # bf16 momentum: narrowed back (exact)
                    items.append((self.ck[idx, j, :n], None, buf[b:b + n]))
                else:
                    items.append((self.ck[idx, j, :n], buf[b:b + n],
                                  self.p16[b:b + n] if j == 0 else None))
            self._pending_init.discard(slot)
            cfg = MemberConfig(**meta["config"])
            self.members[slot] = cfg
            self._write_hp(slot, cfg, int(meta["t"]))
        multi_copy(items)
        self._dirty = True

    def pool_state(self, meta: dict) -> dict:
        """A pool checkpoint in the ``slot_state`` format (views, no copy)."""
        n, idx = meta["n"], meta["ck"]
        st = {"config": meta["config"], "t": meta["t"], "p32": self.ck[idx, 0, :n],
              "m32": self.ck[idx, 1, :n], "optimizer": self.optimizer}
        if self.optimizer == "adamw":
            st["v32"] = self.ck[idx, 2, :n]
        return st

    # -- flat checkpoint images (C4: point-to-point copies between ranks) ----------------------
    def _n_state_buffers(self) -> int:
        return 3 if self.optimizer == "adamw" else 2

    def empty_packed_state(self, width: int) -> torch.Tensor:
        n = self.used_params_for(width)
        return torch.empty(2 + self._n_state_buffers() * n, dtype=torch.float32,
                           device=self.device)

    def pack_state(self, state: dict) -> torch.Tensor:
        """[t, seed (int32 bit patterns), p32, m32(, v32)] as one f32 tensor."""
        head = torch.tensor([int(state["t"]), int(state["config"]["seed"])], dtype=torch.int32)
        parts = [head.view(torch.float32).to(self.device), state["p32"], state["m32"]]
        if self.optimizer == "adamw":
            parts.append(state["v32"])
        return torch.cat([t.reshape(-1).to(self.device, torch.float32) for t in parts])

    def unpack_state(self, buf: torch.Tensor, width: int) -> dict:
        n = self.used_params_for(width)
        t, seed = (int(v) for v in buf[:2].view(torch.int32).cpu().tolist())
        st = {"config": MemberConfig(width=width, lr=0.0, seed=seed).to_dict(), "t": t,
              "p32": buf[2:2 + n], "m32": buf[2 + n:2 + 2 * n], "optimizer": self.optimizer}
        if self.optimizer == "adamw":
            st["v32"] = buf[2 + 2 * n:2 + 3 * n]
        return st

    def slot_state(self, slot: int, to_cpu: bool = False) -> dict:
        """Device checkpoint of a member: config, step count, weights and optimizer state
        (only the used prefix of the slot region is copied)."""
        self._run_pending_init()
        self._join()
        b = self.slot_base(slot)
        reg = slice(b, b + self.used_params(slot))
        mv = (lambda t: t.detach().cpu().clone()) if to_cpu else (lambda t: t.detach().clone())
        st = {"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
              "p32": mv(self.master(slot)), "m32": mv(self.m32[reg]),
              "optimizer": self.optimizer}
        if self.optimizer == "adamw":
            st["v32"] = mv(self.v32[reg])
        return st

    def load_slot_state(self, slot: int, state: dict) -> None:
        self._join()
        self._pending_init.discard(slot)
        cfg = MemberConfig(**state["config"])
        self.members[slot] = cfg
        self._write_hp(slot, cfg, int(state["t"]))
        b = self.slot_base(slot)
        reg = slice(b, b + state["p32"].numel())
        self._set_master(b, state["p32"])
        self.m32[reg].copy_(state["m32"])
        if self.optimizer == "adamw":
            self.v32[reg].copy_(state["v32"])
        self._dirty = True

    def copy_member(self, src: int, dst: int, **hp_changes) -> None:
        """PBT exploit inside one device: dst <- src (weights, optimizer state, step count)."""
        self._run_pending_init()
        self._join()
        self._pending_init.discard(dst)
        rs, rd = self._region(src), self._region(dst)
        if self.split:
            self.plo[rd].copy_(self.plo[rs])
        else:
            self.p32[rd].copy_(self.p32[rs])
        self.p16[rd].copy_(self.p16[rs])
        self.m32[rd].copy_(self.m32[rs])
        if self.optimizer == "adamw":
            self.v32[rd].copy_(self.v32[rs])
        cfg = dataclasses.replace(self.members[src], **hp_changes)
        self._check_member(cfg)
        self.members[dst] = cfg
        self._write_hp(dst, cfg, int(self.hp[src]["t"]))
        self._dirty = True

    # ------------------------------------------------------------------ tables
    def _build_tables(self, rows: int, member_rows: bool = False) -> dict:
        """Trial-layer descriptors + per-layer work lists, built with numpy (no per-item loops).
        ``rows``: the launch's rows (buffer layout); with ``member_rows`` each trial-layer uses
        its member's own batch (train), else all ``rows`` (evaluation)."""
        L = self.L
        tl = np.zeros(self.capacity * L, dtype=TL_DTYPE)
        act_slot = rows * self.act_row
        layer_base = (np.concatenate([[0], np.cumsum(self.nmax)]) * rows).astype(np.int64)
        slots = np.array(self.active_slots(), dtype=np.int64)
        fwd: List[np.ndarray] = []
        bwd: List[np.ndarray] = []
        bwd0f = np.zeros((0, 2), np.int32)
        if len(slots):
            widths = np.array([self.members[s].width for s in slots])
            used = (np.array([self.member_rows(self.members[s]) for s in slots], dtype=np.int64)
                    if member_rows else np.full(len(slots), rows, dtype=np.int64))
            # per-slot layer dims / offsets (vectorised over slots, looped over the few layers)
            wp = (widths + TILE - 1) // TILE * TILE
            Ks, Ns = [], []
            for l in range(L):
                K = np.full_like(wp, self.K0) if l == 0 else wp
                N = np.full_like(wp, TILE) if l == L - 1 else wp
                Ks.append(K)
                Ns.append(N)
            off = np.zeros_like(wp)
            for l in range(L):
                K, N = Ks[l], Ns[l]
                i = slots * L + l
                w_off = slots * self.slot_params + off
                b_off = w_off + (K * N + TILE - 1) // TILE * TILE
                off = off + (K * N + TILE - 1) // TILE * TILE + (N + TILE - 1) // TILE * TILE
                y_off = slots * act_slot + layer_base[l]
                prev = slots * act_slot + layer_base[l - 1] if l > 0 else np.zeros_like(slots)
                tl["K"][i] = K
                tl["N"][i] = N
                tl["trial"][i] = slots
                # real extents: the kernels skip the dead padding's HBM traffic (pop_mlp.hip)
                tl["n_real"][i] = self.num_classes if l == L - 1 else widths
                tl["k_real"][i] = self.in_features if l == 0 else widths
                tl["w_off"][i] = w_off
                tl["b_off"][i] = b_off
                tl["x_off"][i] = prev
                tl["y_off"][i] = y_off
                tl["gx_off"][i] = prev if l > 0 else -1
                tl["rows"][i] = used
                tn = self.fwd_tn if l < L - 1 else TILE   # the loss layer: one 64-wide tile
                nt, nk = -(-N // tn), K // TILE    # a 128-wide tiling ends in a 64-wide tile
                # a forward tile costs ~K, a backward k-strip ~N
                fwd.append(_work_list(np.repeat(i, nt), _ranges(nt), np.repeat(K, nt)))
                bwd.append(_work_list(np.repeat(i, nk), _ranges(nk), np.repeat(N, nk)))
                if l == 0 and L >= 2:
                    # the fused first layer (backward of step t + forward of step t + 1,
                    # csrc/pop_mlp.hip mlp_bwd0_fwd_kernel): one item per 64-row chunk of W0,
                    # each walking all of K
                    nc = N // TILE
                    bwd0f = _work_list(np.repeat(i, nc), _ranges(nc), np.repeat(K, nc))
        else:
            fwd = [np.zeros((0, 2), np.int32) for _ in range(L)]
            bwd = [np.zeros((0, 2), np.int32) for _ in range(L)]
        out = {"tl_np": tl, "rows": rows, "fwd_np": fwd, "bwd_np": bwd, "fwd_tn": self.fwd_tn,
               "bwd0f_np": bwd0f}
        self._validate_tables(tl, fwd, bwd, rows, bwd0f)
        if self.device.type == "cuda":
            from ._lib import upload, upload_bytes
            out["tl"] = upload_bytes(tl, self.device)
            out["fwd"] = [upload(w, self.device) for w in fwd]
            out["bwd"] = [upload(w, self.device) for w in bwd]
            out["bwd0f"] = upload(bwd0f, self.device) if len(bwd0f) else None
        out["n_fwd"] = [len(w) for w in fwd]
        out["n_bwd"] = [len(w) for w in bwd]
        out["n_bwd0f"] = len(bwd0f)
        return out

    def _validate_tables(self, tl, fwd, bwd, rows, bwd0f=None) -> None:
        """Bounds check of every descriptor a launch will read (SURVEY §5 "race detection /
        sanitizers"): the kernels index memory only through these tables, so a table that
        passes here cannot make a kernel read or write outside its buffers.  Vectorised over
        the table (microseconds per refresh), always on."""
        L = self.L
        n_tl = len(tl)
        params = self.capacity * self.slot_params
        act = self.capacity * rows * self.act_row
        live = tl["K"] > 0
        t = tl[live]
        bad = []
        if ((t["K"] % TILE) | (t["N"] % TILE)).any():
            bad.append("K/N not multiples of 64")
        if (t["w_off"] < 0).any() or (t["w_off"] + t["K"].astype(np.int64) * t["N"] > params).any():
            bad.append("weights outside the parameter buffers")
        if (t["b_off"] < 0).any() or (t["b_off"] + t["N"] > params).any():
            bad.append("bias outside the parameter buffers")
        first = (np.flatnonzero(live) % L) == 0
        xin = t[~first]
        if (xin["x_off"] < 0).any() or (xin["x_off"] + rows * xin["K"].astype(np.int64) > act).any():
            bad.append("layer input outside the activation buffer")
        if (t["K"][first] != self.K0).any():
            bad.append("first layer K differs from the input width")
        if (t["y_off"] < 0).any() or (t["y_off"] + rows * t["N"].astype(np.int64) > act).any():
            bad.append("layer output outside the activation buffer")
        if (t["rows"] < 128).any() or (t["rows"] % 128).any() or (t["rows"] > rows).any():
            bad.append("trial rows outside the launch's row blocks")
        if (t["n_real"] > t["N"]).any() or (t["k_real"] > t["K"]).any() or \
                (t["n_real"] < 1).any() or (t["k_real"] < 1).any() or (t["trial"] < 0).any() or \
                (t["trial"] >= self.capacity).any():
            bad.append("trial / class fields out of range")
        fused = [("bwd0f", [bwd0f], "N")] if bwd0f is not None and len(bwd0f) else []
        for name, lists, per in [("fwd", fwd, "N"), ("bwd", bwd, "K")] + fused:
            for l, w in enumerate(lists):
                if not len(w):
                    continue
                w = w[w[:, 0] != -1]          # padding entries (no-op workgroups)
                if not len(w):
                    continue
                idx = w[:, 0]
                if (idx < 0).any() or (idx >= n_tl).any() or not live[idx].all():
                    bad.append(f"{name} work item names a missing trial-layer")
                    break
                if name == "bwd0f" and (idx % L != 0).any():
                    bad.append("fused first-layer item names another layer")
                    break
                tile = self.fwd_tn if (name == "fwd" and l < L - 1) else TILE
                if (w[:, 1] < 0).any() or (w[:, 1] >= -(-tl[per][idx] // tile)).any():
                    bad.append(f"{name} work item tile out of range")
                    break
        if bad:
            raise ValueError("population work tables fail the bounds check: " + "; ".join(bad))

    def _refresh(self) -> None:
        self._run_pending_init()
        if not self._dirty:
            return
        self._join()
        self._tables = {"train": self._build_tables(self.batch_size, member_rows=True)}
        # per-slot train rows (the loss statistics are sums over them); eval: built lazily
        self._rows_np = np.array([self.member_rows(m) if m is not None else self.batch_size
                                  for m in self.members], dtype=np.float64)
        if self.device.type == "cuda":
            self._upload_hp()
        self._active_np = np.array([m is not None for m in self.members])
        from ._lib import upload
        self._active_t = upload(self._active_np.astype(np.int32), self.device)
        self._any_dropout = any(m is not None and m.dropout > 0 for m in self.members)
        if self.backend == "hip":
            tb = self._tables["train"]
            self._parts = self._partition(tb)
            self._ptr = {"plo": self.plo.data_ptr(), "p16": self.p16.data_ptr(),
                         "m32": self.m32.data_ptr(), "v32": self.v32.data_ptr(),
                         "act": self.act.data_ptr(), "grad": self.grad.data_ptr(),
                         "hp": self.hp_dev.data_ptr(), "loss": self.loss.data_ptr(),
                         "correct": self.correct.data_ptr(), "tl": tb["tl"].data_ptr(),
                         "fwd": [w.data_ptr() for w in tb["fwd"]],
                         "bwd": [w.data_ptr() for w in tb["bwd"]]}
            # (the fused first layer's work list lives in each part)
            for part in self._parts:
                part["step"] = self._step_args(part)
        self._dirty = False

    def _step_args(self, part) -> "_MlpStep":
        """``mopt_mlp_step`` argument block of one trial group (pointers of this refresh)."""
        P, L = self._ptr, self.L
        a = _MlpStep()
        a.tls = P["tl"]
        for l in range(L):
            a.fwd[l], a.bwd[l] = part["fwd"][l], part["bwd"][l]
            a.n_fwd[l], a.n_bwd[l] = part["n_fwd"][l], part["n_bwd"][l]
        a.L, a.rb, a.drop = L, self.batch_size // 128, int(self._any_dropout)
        a.n_stats = self.capacity      # > 1 row block: the step zeroes loss/correct first
        a.fwd_tn = self.fwd_tn
        a.narrow = int(self.num_classes <= NARROW_CLASSES)
        a.opt = 2 if self.momentum_dtype == "bf16" else OPTIMIZERS[self.optimizer]
        for n in ("plo", "p16", "m32", "v32", "act", "grad", "hp", "loss", "correct"):
            setattr(a, n, P[n])
        a.bwd0f = part["bwd0f"] or 0
        a.n_bwd0f = part["n_bwd0f"]
        a.fuse0 = int(self.fuse_first_layer)
        a.inv_b = -1.0                 # the mean over each trial's own rows
        part["step_ptr"] = ctypes.addressof(a)
        return a

    def _join(self) -> None:
        """Order the main stream after every side stream's queued work (no host wait)."""
        self._fork_needed = True
        if not self._side_pending:
            return
        main = torch.cuda.current_stream(self.device)
        for i, side in enumerate(self._side_streams[:len(self._parts) - 1]):
            ev = self._events[i + 1]
            ev.record(side)
            main.wait_event(ev)
        self._side_pending = False

    def _partition(self, tb: dict) -> list:
        """Split the train work lists into ``n_streams`` groups of trials with equal padded
        parameter counts (greedy, heaviest first); each keeps its LPT order.  Returns one
        ``{"fwd": [ptr per layer], "bwd": [...], "n_fwd": [...], "n_bwd": [...]}`` per group."""
        slots = self.active_slots()
        n = min(self.n_streams, max(1, len(slots)))
        if self.batch_size > 128:
            n = 1   # the step's stats zeroing covers every trial: one stream orders it
        if n <= 1:
            b0f = tb.get("bwd0f")
            return [{"fwd": [w.data_ptr() for w in tb["fwd"]],
                     "bwd": [w.data_ptr() for w in tb["bwd"]],
                     "n_fwd": tb["n_fwd"], "n_bwd": tb["n_bwd"],
                     "bwd0f": b0f.data_ptr() if b0f is not None else None,
                     "n_bwd0f": tb["n_bwd0f"]}]
        from ._lib import upload
        cost = {s: self.padded_params(s) for s in slots}
        load = [0] * n
        part_of = np.full(self.capacity, -1, dtype=np.int64)
        for s in sorted(slots, key=lambda s: -cost[s]):
            p = min(range(n), key=load.__getitem__)
            part_of[s] = p
            load[p] += cost[s]
        L = self.L
        parts = []
        keep = []
        for p in range(n):
            fwd = [_reschedule(w, part_of, p, L, tb["tl_np"], "K") for w in tb["fwd_np"]]
            bwd = [_reschedule(w, part_of, p, L, tb["tl_np"], "N") for w in tb["bwd_np"]]
            fwd_t = [upload(w, self.device) for w in fwd]
            bwd_t = [upload(w, self.device) for w in bwd]
            keep += fwd_t + bwd_t
            b0f = (_reschedule(tb["bwd0f_np"], part_of, p, L, tb["tl_np"], "K")
                   if len(tb["bwd0f_np"]) else np.zeros((0, 2), np.int32))
            b0f_t = upload(b0f, self.device) if len(b0f) else None
            if b0f_t is not None:
                keep.append(b0f_t)
            parts.append({"fwd": [w.data_ptr() for w in fwd_t],
                          "bwd": [w.data_ptr() for w in bwd_t],
                          "n_fwd": [len(w) for w in fwd], "n_bwd": [len(w) for w in bwd],
                          "bwd0f": b0f_t.data_ptr() if b0f_t is not None else None,
                          "n_bwd0f": len(b0f)})
        tb["parts_keep"] = keep           # the work lists live as long as the table
        while len(self._side_streams) < n - 1:
            self._side_streams.append(torch.cuda.Stream(device=self.device))
        while len(self._events) < n:
            self._events.append(torch.cuda.Event())
        return parts

    # ------------------------------------------------------------------ training
    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """One SGD/AdamW step of every active member on the shared minibatch (x [B,K0] bf16, y [B])."""
        self._refresh()
        if x.shape != (self.batch_size, self.K0):
            raise ValueError(f"x must be [{self.batch_size}, {self.K0}] (padded), got {tuple(x.shape)}")
        self.hp["t"][self._active_np] += 1
        if self.backend == "hip":
            self._train_step_hip(x, y)     # advances the device step counters itself
        else:
            self._train_step_torch(x, y)

    def train_steps(self, batches) -> None:
        """``len(batches)`` consecutive steps (``batches`` = [(x, y)] of the interval): on the
        HIP backend one host call per trial group queues them all (``mopt_mlp_steps``), so the
        per-step host cost is the kernel launches alone; otherwise :meth:`train_step` each."""
        if self.backend != "hip" or _lib_sync_check() or len(batches) <= 1:
            for x, y in batches:
                self.train_step(x, y)
            return
        self._refresh()
        n = len(batches)
        xs = np.empty(n, dtype=np.uint64)
        ys = np.empty(n, dtype=np.uint64)
        keep = []
        for i, (x, y) in enumerate(batches):
            if x.shape != (self.batch_size, self.K0):
                raise ValueError(f"x must be [{self.batch_size}, {self.K0}] (padded), got "
                                 f"{tuple(x.shape)}")
            if y.shape != (self.batch_size,) or y.dtype != torch.int32:
                raise ValueError(f"y must be [{self.batch_size}] int32, got {tuple(y.shape)} "
                                 f"{y.dtype}")
            if not x.is_contiguous():
                x = x.contiguous()
                keep.append(x)
            if not y.is_contiguous():
                y = y.contiguous()
                keep.append(y)
            xs[i], ys[i] = x.data_ptr(), y.data_ptr()
        self.hp["t"][self._active_np] += n
        from ._lib import check
        lib, main = self._lib, torch.cuda.current_stream(self.device)
        parts = self._parts
        if len(parts) > 1:
            if self._fork_needed:
                ev = self._events[0]
                ev.record(main)
                for side in self._side_streams[:len(parts) - 1]:
                    side.wait_event(ev)
                self._fork_needed = False
            self._side_pending = True
        streams = [main if i == 0 else self._side_streams[i - 1] for i in range(len(parts))]
        chunk = self.step_chunk if len(parts) > 1 and self.step_chunk > 0 else n
        # the groups' steps are queued round-robin, ``chunk`` at a time: all streams busy from
        # the interval's start to its end (mopt_mlp_steps_range keeps the fused first layer
        # across the runs)
        for c0 in range(0, n, chunk):
            cnt = min(chunk, n - c0)
            for part, stream in zip(parts, streams):
                check(lib.mopt_mlp_steps_range(part["step_ptr"], xs.ctypes.data, ys.ctypes.data,
                                               c0, n, cnt, stream.cuda_stream), "mlp_steps")
        for stream in streams[1:]:  # temporaries are freed on return: not before a side stream
            for t in keep:          # read them
                t.record_stream(stream)

    def _train_step_hip(self, x, y) -> None:
        from ._lib import check
        lib, tb, P = self._lib, self._tables["train"], self._ptr
        main = torch.cuda.current_stream(self.device)
        # one 128-row block per trial: the loss kernel stores the statistics (no zero-fill) and
        # advances the device step counters; the hidden layers run before it, so they key their
        # dropout masks with t + 1 (the step being taken).  More row blocks: the step zeroes the
        # statistics and the loss kernel adds into them.
        rb = self.batch_size // 128
        xp = x.data_ptr() if x.is_contiguous() else x.contiguous().data_ptr()
        parts = self._parts
        if len(parts) > 1:
            if self._fork_needed:
                # fork: the side streams follow everything queued on the main stream so far
                ev = self._events[0]
                ev.record(main)
                for side in self._side_streams[:len(parts) - 1]:
                    side.wait_event(ev)
                self._fork_needed = False
            self._side_pending = True
        for i, part in enumerate(parts):
            stream = main if i == 0 else self._side_streams[i - 1]
            self._launch_step(lib, P, part, xp, y.data_ptr(), rb, stream.cuda_stream, check)

    def _launch_step(self, lib, P, part, xp, yp, rb, stream, check) -> None:
        """The 2L launches of one train step for one group of trials on ``stream``: one host
        call (``mopt_mlp_step``), or one call per kernel under MOPT_SYNC_CHECK (each launch
        checked by name)."""
        if not _lib_sync_check():
            check(lib.mopt_mlp_step(part["step_ptr"], xp, yp, stream), "mlp_step")
            return
        L = self.L
        narrow = self.num_classes <= NARROW_CLASSES
        ce_flags = FWD_WRITE_GRAD | FWD_COUNT_STEP | (FWD_STORE_STATS if rb == 1 else 0) | \
            (FWD_NARROW_CE if narrow else 0)
        if rb != 1:
            self.stats[:2 * self.capacity].zero_()
        drop = self._any_dropout
        act, tl = P["act"], P["tl"]
        for l in range(L - 1):
            check(lib.mopt_mlp_fwd(tl, part["fwd"][l], part["n_fwd"][l], rb, xp if l == 0 else act,
                                   P["plo"], P["p16"], act, P["hp"], 1, l,
                                   FWD_RELU | (FWD_DROPOUT if drop else 0), self.fwd_tn, stream),
                  "mlp_fwd")
        check(lib.mopt_mlp_fwd_ce(tl, part["fwd"][L - 1], part["n_fwd"][L - 1], rb,
                                  xp if L == 1 else act, P["plo"], P["p16"], yp,
                                  P["grad"], P["loss"], P["correct"], P["hp"],
                                  -1.0, ce_flags, stream), "mlp_fwd_ce")
        opt = 2 if self.momentum_dtype == "bf16" else OPTIMIZERS[self.optimizer]
        for l in range(L - 1, -1, -1):
            flags = BWD_UPDATE_BIAS | (BWD_NARROW if (narrow and l == L - 1) else 0)
            if l > 0:
                flags |= BWD_HAS_DX | (BWD_IN_DROPOUT if drop else 0)
            check(lib.mopt_mlp_bwd(tl, part["bwd"][l], part["n_bwd"][l], xp if l == 0 else act,
                                   P["grad"], P["plo"], P["p16"], P["m32"], P["v32"], P["hp"],
                                   opt, flags, rb, stream), "mlp_bwd")

    def _train_step_torch(self, x, y) -> None:
        self.stats.zero_()
        em = self.emulate_bf16
        for s in self.active_slots():
            cfg = self.members[s]
            rows = self.member_rows(cfg)
            xf, ys = x[:rows].float(), y[:rows]
            t = int(self.hp[s]["t"])
            layers = self.layer_views(s)
            mom = self.layer_views(s, self.m32)
            acts = [xf]
            a = xf
            for l in range(self.L - 1):
                w, b = layers[l]
                a = ref.hidden_fwd(a, w, b, cfg.dropout, cfg.seed, l, t, emulate_bf16=em)
                acts.append(a)
            w, b = layers[-1]
            wq = ref.bf16_weight(w) if em else w
            logits = a @ wq.t() + b
            ls, cs, dz = ref.softmax_ce(logits, ys, self.num_classes, 1.0 / rows, em)
            self.loss[s] = ls
            self.correct[s] = cs
            inv_keep = ref._inv_keep(cfg.dropout) if cfg.dropout > 0 else 1.0
            for l in range(self.L - 1, -1, -1):
                w, b = layers[l]
                a_in = acts[l]
                dw = dz.t() @ a_in
                db = dz.sum(0)
                if l > 0:
                    wq = ref.bf16_weight(w) if em else w
                    dx = dz @ wq
                    dz_prev = torch.where(a_in > 0, dx * inv_keep, torch.zeros_like(dx))
                    dz_prev = ref.bf16_round(dz_prev) if em else dz_prev
                mw, mb = mom[l]
                if self.optimizer == "sgd":
                    ref.sgd_update(w, mw, dw, cfg.lr, cfg.momentum, cfg.weight_decay)
                    ref.sgd_update(b, mb, db, cfg.lr, cfg.momentum, 0.0)
                else:
                    vw, vb = self.layer_views(s, self.v32)[l]
                    ref.adamw_update(w, mw, vw, dw, cfg.lr, cfg.momentum, cfg.beta2, cfg.eps,
                                     cfg.weight_decay, t)
                    ref.adamw_update(b, mb, vb, db, cfg.lr, cfg.momentum, cfg.beta2, cfg.eps, 0.0, t)
                if l > 0:
                    dz = dz_prev
            reg = self._region(s)
            self.p16[reg] = ref.split_f32(self.p32[reg])[0]

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, x: torch.Tensor, y: torch.Tensor, slots=None):
        """Mean loss and accuracy per slot (numpy [capacity]; NaN for empty slots and for slots
        outside ``slots`` when a subset is given)."""
        handle = self.evaluate_async(x, y, slots)
        return self.eval_result(self.stats_snapshot(), handle)

    @torch.no_grad()
    def evaluate_async(self, x: torch.Tensor, y: torch.Tensor, slots=None):
        """Queue the evaluation kernels (no host sync); read back with :meth:`eval_result`."""
        self._refresh()
        rows = x.shape[0]
        subset = None if slots is None else set(int(s) for s in slots)
        if rows % 128 or rows > self.eval_batch:
            raise ValueError(f"eval rows must be a multiple of 128 and <= {self.eval_batch}")
        handle = {"rows": rows, "subset": subset}
        self._join()
        if self.backend == "hip":
            from ._lib import check, stream_ptr
            if "eval" not in self._tables:
                self._tables["eval"] = self._build_tables(self.eval_batch)
            lib, tb, L = self._lib, self._tables["eval"], self.L
            if subset is not None:
                tb = self._subset_table(tb, subset)
            handle["table"] = tb  # keeps the subset work lists alive until the kernels ran
            stream = stream_ptr(self.device)
            self.stats[2 * self.capacity:].zero_()
            xb = x.contiguous()
            rb = rows // 128
            for l in range(L - 1):
                src = xb if l == 0 else self.act_eval
                check(lib.mopt_mlp_fwd(tb["tl"].data_ptr(), tb["fwd"][l].data_ptr(), tb["n_fwd"][l],
                                       rb, src.data_ptr(), self.plo.data_ptr(), self.p16.data_ptr(),
                                       self.act_eval.data_ptr(), self.hp_dev.data_ptr(), 0, l,
                                       FWD_RELU, tb["fwd_tn"], stream), "mlp_fwd(eval)")
            src = xb if L == 1 else self.act_eval
            check(lib.mopt_mlp_fwd_ce(tb["tl"].data_ptr(), tb["fwd"][L - 1].data_ptr(),
                                      tb["n_fwd"][L - 1], rb, src.data_ptr(), self.plo.data_ptr(),
                                      self.p16.data_ptr(), y.data_ptr(), self.grad.data_ptr(),
                                      self.eval_loss.data_ptr(), self.eval_correct.data_ptr(),
                                      self.hp_dev.data_ptr(), 1.0,
                                      FWD_NARROW_CE if self.num_classes <= NARROW_CLASSES else 0,
                                      stream), "mlp_fwd_ce(eval)")
        else:
            self.stats[2 * self.capacity:].zero_()
            xf = x.float()
            em = self.emulate_bf16
            for s in self.active_slots():
                if subset is not None and s not in subset:
                    continue
                cfg = self.members[s]
                layers = self.layer_views(s)
                a = xf
                for l in range(self.L - 1):
                    w, b = layers[l]
                    a = ref.hidden_fwd(a, w, b, cfg.dropout, cfg.seed, l, 0, emulate_bf16=em,
                                       train=False)
                w, b = layers[-1]
                wq = ref.bf16_weight(w) if em else w
                ls, cs, _ = ref.softmax_ce(a @ wq.t() + b, y, self.num_classes, 1.0, em)
                self.eval_loss[s] = ls
                self.eval_correct[s] = cs
        return handle

    def device_busy(self):
        """A callable that stays True while the work queued so far is still running on the GPU
        (always True on the CPU backend, where nothing runs asynchronously)."""
        self._join()
        return device_busy(self.device)

    def stats_snapshot(self) -> np.ndarray:
        """One device->host copy of the train and eval statistics (waits for queued work)."""
        self._join()
        return self.stats.cpu().numpy().reshape(4, self.capacity)

    def stats_snapshot_async(self) -> StatsSnapshot:
        self._join()
        return StatsSnapshot(self.stats, self.capacity, self._rows_np.copy())

    def raw_results(self, snap: np.ndarray, handle, rows=None):
        """(train loss, eval loss, eval accuracy) per slot from a snapshot, unmasked: the slots
        may have been re-assigned since the snapshot was queued (``rows``: the per-slot train
        rows of that time, ``StatsSnapshot.rows``; default the current ones)."""
        tl = snap[0].astype(np.float64) / (self._rows_np if rows is None else rows)
        if handle is None:
            nan = np.full(self.capacity, np.nan)
            return tl, nan, nan
        rows = handle["rows"]
        return tl, snap[2].astype(np.float64) / rows, snap[3].astype(np.float64) / rows

    def eval_result(self, snap: np.ndarray, handle):
        rows, subset = handle["rows"], handle["subset"]
        loss = snap[2].astype(np.float64) / rows
        acc = snap[3].astype(np.float64) / rows
        for s in range(self.capacity):
            if self.members[s] is None or (subset is not None and s not in subset):
                loss[s] = np.nan
                acc[s] = np.nan
        return loss, acc

    def train_loss(self, snap: Optional[np.ndarray] = None) -> np.ndarray:
        """Mean training loss of the last step per slot."""
        snap = self.stats_snapshot() if snap is None else snap
        out = snap[0].astype(np.float64) / self._rows_np
        out[~np.array([m is not None for m in self.members])] = np.nan
        return out

    def _subset_table(self, tb: dict, subset) -> dict:
        L = self.L
        keep = np.zeros(self.capacity, dtype=bool)
        keep[list(subset)] = True
        out = dict(tb)
        fwd = [_reschedule(w, keep.astype(np.int64), 1, L, tb["tl_np"], "K")
               for w in tb["fwd_np"]]
        from ._lib import upload
        out["fwd"] = [upload(w, self.device) for w in fwd]
        out["n_fwd"] = [len(w) for w in fwd]
        return out

