"""Llama-style decoder LMs trained as device populations (BASELINE.json configs 4 and 5).

``PopulationLM`` keeps ``capacity`` trials of ONE architecture on a GPU.  Every parameter tensor
is stacked over the population (``[P, ...]``), so a step is a handful of batched launches
regardless of ``P``:

* GEMMs: ``torch.bmm`` over the population dimension (hipBLASLt strided-batched: plain library
  GEMMs, the one place we do not hand-write the kernel);
* embedding gather/scatter, RMSNorm, RoPE + head split, causal flash attention, SwiGLU, the
  vocabulary cross-entropy and the per-trial fused AdamW: hand-written gfx950 kernels
  (:mod:`metaopt_amd.ops.lm`);
* parameters live in flat buffers -- bf16 working copy ``p16`` (autograd leaves are views of it,
  with their ``.grad`` pre-bound to views of the flat bf16 gradient ``g16``), f32 master ``p32``,
  AdamW moments ``m``/``v`` -- so the optimizer is ONE fused kernel over all tensors and trials,
  and a checkpoint / PBT exploit copy of a trial is a fixed set of contiguous slices.

The member interface (``set_member``, ``update_hparams``, ``save_states``/``load_states``,
``evaluate_async``, ...) is the one :class:`~metaopt_amd.worker.population_sweep.PopulationSweep`
drives for the MLP population, so the same sweep runs ASHA / PBT / TPE over LMs.

Presets: ``llama-125m`` (d 768, 12 layers, 12 heads, SwiGLU 2048, vocab 32000; ~134M params with
an untied head) and ``tiny-2layer`` (the 2-layer LM of config 4).
"""
from __future__ import annotations

import dataclasses
import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import lm as ops
from ..ops.population import MemberConfig

HP_T = np.dtype([("t", "<i4")])


@dataclass
class LMConfig:
    vocab: int = 32000
    d_model: int = 768
    n_layers: int = 12
    n_heads: int = 12
    ffn: int = 2048
    seq_len: int = 512
    rope_base: float = 10000.0
    norm_eps: float = 1e-5
    init_std: float = 0.02

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads


PRESETS = {
    "llama-125m": LMConfig(),
    "tiny-2layer": LMConfig(vocab=4096, d_model=256, n_layers=2, n_heads=4, ffn=704,
                            seq_len=256),
    "micro": LMConfig(vocab=512, d_model=128, n_layers=2, n_heads=2, ffn=256, seq_len=64),
}


def param_specs(cfg: LMConfig):
    """(name, per-trial shape, init) of every tensor; init = ('normal', std) or ('ones',)."""
    d, F, V, L = cfg.d_model, cfg.ffn, cfg.vocab, cfg.n_layers
    out_std = cfg.init_std / math.sqrt(2 * L)
    specs = [("embed", (V, d), ("normal", cfg.init_std))]
    for l in range(L):
        specs += [(f"l{l}.attn_norm", (d,), ("ones",)),
                  (f"l{l}.wqkv", (d, 3 * d), ("normal", cfg.init_std)),
                  (f"l{l}.wo", (d, d), ("normal", out_std)),
                  (f"l{l}.mlp_norm", (d,), ("ones",)),
                  (f"l{l}.wgu", (d, 2 * F), ("normal", cfg.init_std)),
                  (f"l{l}.wdown", (F, d), ("normal", out_std))]
    specs += [("final_norm", (d,), ("ones",)), ("head", (d, V), ("normal", cfg.init_std))]
    return specs


class PopulationLM:
    def __init__(self, capacity: int, config="tiny-2layer", batch_size: int = 8,
                 seq_len: Optional[int] = None, device="cuda", max_grad_norm: float = 1.0,
                 eval_batch: Optional[int] = None):
        self.cfg = PRESETS[config] if isinstance(config, str) else config
        if seq_len is not None:
            self.cfg = dataclasses.replace(self.cfg, seq_len=seq_len)
        c = self.cfg
        if c.head_dim != 64 or c.seq_len % 64:
            raise ValueError("the attention kernel needs head_dim 64 and seq_len % 64 == 0")
        self.device = torch.device(device)
        self.backend = "hip" if self.device.type == "cuda" else "torch"
        self.capacity = P = int(capacity)
        self.batch_size = int(batch_size)          # sequences per trial per step
        self.eval_batch = int(eval_batch or batch_size)
        self.tokens_per_step = self.batch_size * c.seq_len
        self.max_grad_norm = float(max_grad_norm)
        self.specs = param_specs(c)
        self.segments = []
        off = 0
        for _, shape, _ in self.specs:
            n = int(np.prod(shape))
            self.segments.append((off, n))
            off += P * n
        self.n_flat = off
        dev = self.device
        self.p32 = torch.zeros(off, dtype=torch.float32, device=dev)
        self.p16 = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        self.g16 = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        self.m = torch.zeros(off, dtype=torch.float32, device=dev)
        self.v = torch.zeros(off, dtype=torch.float32, device=dev)
        self.W: Dict[str, torch.Tensor] = {}
        for (name, shape, _), (o, n) in zip(self.specs, self.segments):
            leaf = self.p16[o:o + P * n].view(P, *shape)
            leaf.requires_grad_(True)
            leaf.grad = self.g16[o:o + P * n].view(P, *shape)
            self.W[name] = leaf
        self.cos, self.sin = ops.rope_tables(c.seq_len, c.rope_base, device=dev)
        self.opt = ops.FlatAdamW(self.segments, P, dev)
        self.hp = np.zeros(P, dtype=[("t", "<i4")])
        self.lm_hp = np.zeros(P, dtype=ops.LM_HP_DTYPE)
        self.members: List[Optional[MemberConfig]] = [None] * P
        self.stats = torch.zeros(4 * P, dtype=torch.float32, device=dev)
        self._ck = None

    # ------------------------------------------------------------------ members
    @property
    def n_params(self) -> int:
        return sum(n for _, n in self.segments)

    def active_slots(self):
        return [s for s, m in enumerate(self.members) if m is not None]

    def _write_hp(self, slot, cfg: MemberConfig, t: int):
        self.hp[slot]["t"] = t
        self.lm_hp[slot] = (cfg.lr, cfg.momentum, cfg.beta2, cfg.eps, cfg.weight_decay,
                            self.max_grad_norm, t, 0)

    def _slices(self, slot):
        return [slice(o + slot * n, o + (slot + 1) * n) for o, n in self.segments]

    def set_member(self, slot: int, cfg: MemberConfig, init: bool = True) -> None:
        self.members[slot] = cfg
        self._write_hp(slot, cfg, 0)
        if not init:
            return
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(cfg.seed) & 0x7FFFFFFF)
        with torch.no_grad():
            for (name, shape, init_), sl in zip(self.specs, self._slices(slot)):
                dst = self.p32[sl]
                if init_[0] == "ones":
                    dst.fill_(1.0)
                else:
                    dst.normal_(0.0, init_[1], generator=gen)
                self.p16[sl] = dst.to(torch.bfloat16)
                self.m[sl].zero_()
                self.v[sl].zero_()

    def update_hparams(self, slot: int, **changes) -> None:
        cfg = dataclasses.replace(self.members[slot], **changes)
        self.members[slot] = cfg
        self._write_hp(slot, cfg, int(self.hp[slot]["t"]))

    def remove_member(self, slot: int) -> None:
        self.members[slot] = None
        self.hp[slot]["t"] = 0
        self.lm_hp[slot] = 0

    def steps_done(self, slot: int) -> int:
        return int(self.hp[slot]["t"])

    # ------------------------------------------------------------------ model
    def _forward(self, tok: torch.Tensor, labels: torch.Tensor, train: bool):
        c, P = self.cfg, self.capacity
        T, d, H = c.seq_len, c.d_model, c.n_heads
        rpt = tok.numel() // P
        R = tok.numel()
        W = self.W
        x = ops.embedding(tok.reshape(-1), W["embed"], rpt)
        for l in range(c.n_layers):
            h = ops.rmsnorm(x, W[f"l{l}.attn_norm"], rpt, c.norm_eps)
            qkv = torch.bmm(h.view(P, rpt, d), W[f"l{l}.wqkv"]).view(R, 3 * d)
            q, k, v = ops.rope_split(qkv, self.cos, self.sin, T, H)
            o = ops.attention(q, k, v)
            x = x + torch.bmm(o.view(P, rpt, d), W[f"l{l}.wo"]).view(R, d)
            h = ops.rmsnorm(x, W[f"l{l}.mlp_norm"], rpt, c.norm_eps)
            gu = torch.bmm(h.view(P, rpt, d), W[f"l{l}.wgu"])
            a = ops.swiglu(gu)
            x = x + torch.bmm(a, W[f"l{l}.wdown"]).view(R, d)
        h = ops.rmsnorm(x, W["final_norm"], rpt, c.norm_eps)
        logits = torch.bmm(h.view(P, rpt, d), W["head"]).view(R, c.vocab)
        if train:
            return ops.cross_entropy(logits, labels.reshape(-1), rpt, grad_scale=1.0 / rpt)
        return ops.ce_eval(logits, labels.reshape(-1), rpt)

    def _expand(self, t: torch.Tensor) -> torch.Tensor:
        """[B, T] shared batch -> [P, B, T] (int32, contiguous)."""
        t = t.to(self.device, torch.int32)
        if t.dim() == 2:
            t = t.unsqueeze(0).expand(self.capacity, *t.shape)
        return t.contiguous()

    def train_step(self, inp: torch.Tensor, tgt: torch.Tensor) -> None:
        """One AdamW step of every member on ``inp``/``tgt`` ([B, T] shared or [P, B, T])."""
        active = np.array([m is not None for m in self.members])
        self.hp["t"][active] += 1
        self.lm_hp["t"] = self.hp["t"]
        self.g16.zero_()
        loss = self._forward(self._expand(inp), self._expand(tgt), train=True)
        loss.sum().backward()
        self.stats[:self.capacity].copy_(loss.detach())
        with torch.no_grad():
            self.opt.step(self.p32, self.p16, self.g16, self.m, self.v, self.lm_hp)

    # ------------------------------------------------------------------ evaluation / stats
    @torch.no_grad()
    def evaluate_async(self, inp, tgt, slots=None):
        loss = self._forward(self._expand(inp), self._expand(tgt), train=False)
        P = self.capacity
        self.stats[2 * P:3 * P].copy_(loss)
        return {"rows": inp.shape[-1] * inp.shape[-2], "subset": None if slots is None
                else set(int(s) for s in slots)}

    def device_busy(self):
        from ..ops.population import device_busy
        return device_busy(self.device)

    def stats_snapshot(self) -> np.ndarray:
        return self.stats.cpu().numpy().reshape(4, self.capacity)

    def train_loss(self, snap=None) -> np.ndarray:
        snap = self.stats_snapshot() if snap is None else snap
        out = snap[0].astype(np.float64) / self.tokens_per_step
        out[[m is None for m in self.members]] = np.nan
        return out

    def eval_result(self, snap, handle):
        loss = snap[2].astype(np.float64) / handle["rows"]
        ppl = np.exp(np.minimum(loss, 50.0))
        for s in range(self.capacity):
            if self.members[s] is None or (handle["subset"] is not None
                                           and s not in handle["subset"]):
                loss[s] = ppl[s] = np.nan
        return loss, ppl

    def evaluate(self, inp, tgt, slots=None):
        return self.eval_result(self.stats_snapshot(), self.evaluate_async(inp, tgt, slots))

    # ------------------------------------------------------------------ checkpoints
    def used_params_for(self, width=None) -> int:
        return self.n_params

    def alloc_ckpt_pool(self, n: int) -> None:
        self._ck = torch.zeros(n, 3, self.n_params, dtype=torch.float32, device=self.device)

    def _gather(self, slot, buf):
        return [buf[sl] for sl in self._slices(slot)]

    @torch.no_grad()
    def save_states(self, pairs) -> list:
        from ..ops.ckpt import multi_copy
        items, metas = [], []
        for slot, idx in pairs:
            for j, buf in enumerate((self.p32, self.m, self.v)):
                o = 0
                for sl in self._slices(slot):
                    n = sl.stop - sl.start
                    items.append((buf[sl], self._ck[idx, j, o:o + n], None))
                    o += n
            metas.append({"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
                          "ck": int(idx), "n": self.n_params})
        multi_copy(items)
        return metas

    @torch.no_grad()
    def load_states(self, pairs) -> None:
        from ..ops.ckpt import multi_copy
        items = []
        for slot, meta in pairs:
            idx = meta["ck"]
            for j, buf in enumerate((self.p32, self.m, self.v)):
                o = 0
                for sl in self._slices(slot):
                    n = sl.stop - sl.start
                    items.append((self._ck[idx, j, o:o + n], buf[sl],
                                  self.p16[sl] if j == 0 else None))
                    o += n
            cfg = MemberConfig(**meta["config"])
            self.members[slot] = cfg
            self._write_hp(slot, cfg, int(meta["t"]))
        multi_copy(items)

    def pool_state(self, meta: dict) -> dict:
        idx = meta["ck"]
        return {"config": meta["config"], "t": meta["t"], "p32": self._ck[idx, 0],
                "m32": self._ck[idx, 1], "v32": self._ck[idx, 2], "optimizer": "adamw"}

    def slot_state(self, slot: int) -> dict:
        cat = lambda buf: torch.cat([buf[sl] for sl in self._slices(slot)])  # noqa: E731
        return {"config": self.members[slot].to_dict(), "t": int(self.hp[slot]["t"]),
                "p32": cat(self.p32), "m32": cat(self.m), "v32": cat(self.v),
                "optimizer": "adamw"}

    @torch.no_grad()
    def load_slot_state(self, slot: int, state: dict) -> None:
        o = 0
        for sl in self._slices(slot):
            n = sl.stop - sl.start
            self.p32[sl] = state["p32"][o:o + n]
            self.m[sl] = state["m32"][o:o + n]
            self.v[sl] = state["v32"][o:o + n]
            self.p16[sl] = self.p32[sl].to(torch.bfloat16)
            o += n
        cfg = MemberConfig(**state["config"])
        self.members[slot] = cfg
        self._write_hp(slot, cfg, int(state["t"]))

    @torch.no_grad()
    def copy_member(self, src: int, dst: int, **hp_changes) -> None:
        """PBT exploit inside one device: dst <- src (weights, moments, step count)."""
        for a, b in zip(self._slices(src), self._slices(dst)):
            for buf in (self.p32, self.p16, self.m, self.v):
                buf[b] = buf[a]
        cfg = dataclasses.replace(self.members[src], **hp_changes)
        self.members[dst] = cfg
        self._write_hp(dst, cfg, int(self.hp[src]["t"]))

    def empty_packed_state(self, width=None) -> torch.Tensor:
        return torch.empty(2 + 3 * self.n_params, dtype=torch.float32, device=self.device)

    def pack_state(self, state: dict) -> torch.Tensor:
        head = torch.tensor([int(state["t"]), int(state["config"]["seed"])], dtype=torch.int32)
        return torch.cat([head.view(torch.float32).to(self.device), state["p32"].reshape(-1),
                          state["m32"].reshape(-1), state["v32"].reshape(-1)])

    def unpack_state(self, buf: torch.Tensor, width=None) -> dict:
        n = self.n_params
        t, seed = (int(v) for v in buf[:2].view(torch.int32).cpu().tolist())
        return {"config": MemberConfig(width=self.cfg.d_model, lr=0.0, seed=seed).to_dict(),
                "t": t, "p32": buf[2:2 + n], "m32": buf[2 + n:2 + 2 * n],
                "v32": buf[2 + 2 * n:], "optimizer": "adamw"}


class SyntheticLM:
    """Token streams from a fixed random sparse bigram model (so the loss can fall well below
    ``log(vocab)``): every token has ``branch`` likely successors.  Pre-generated on the host
    with numpy (vectorised over many chains), stored on the device, sliced per step."""

    def __init__(self, vocab: int, seq_len: int, batch_size: int, n_tokens: int = 1 << 21,
                 branch: int = 8, seed: int = 0, device=None, n_val_seq: Optional[int] = None):
        rng = np.random.default_rng(seed)
        self.vocab, self.seq_len, self.batch_size = vocab, seq_len, batch_size
        succ = rng.integers(0, vocab, size=(vocab, branch))
        probs = rng.dirichlet(np.full(branch, 0.5), size=vocab)
        cdf = np.cumsum(probs, 1)
        L = seq_len + 1
        n_seq = max(batch_size * 4, n_tokens // L)
        toks = np.empty((n_seq, L), dtype=np.int32)
        toks[:, 0] = rng.integers(0, vocab, size=n_seq)
        for t in range(1, L):
            u = rng.random(n_seq)
            prev = toks[:, t - 1]
            k = (u[:, None] > cdf[prev]).sum(1).clip(max=branch - 1)
            toks[:, t] = succ[prev, k]
        dev = torch.device(device) if device is not None else torch.device("cpu")
        n_val = n_val_seq or batch_size
        self.train = torch.from_numpy(toks[n_val:]).to(dev)
        self.val = torch.from_numpy(toks[:n_val]).to(dev)
        self.n_batches = len(self.train) // batch_size

    def batch(self, step: int):
        i = step % self.n_batches
        b = self.train[i * self.batch_size:(i + 1) * self.batch_size]
        return b[:, :-1], b[:, 1:]

    def validation(self):
        return self.val[:, :-1], self.val[:, 1:]


LM_PBT_PRIORS = {
    "/lr": "loguniform(1e-4, 3e-3)",
    "/weight_decay": "loguniform(1e-3, 0.3)",
    "/beta1": "uniform(0.8, 0.95)",
    "/steps": "fidelity(200, 2000, 2)",
}


@dataclass
class LMSweepTask:
    """Maps trial parameters to LM population members (AdamW lr / wd / beta1)."""

    priors: Dict[str, str] = dataclasses.field(default_factory=lambda: dict(LM_PBT_PRIORS))
    fidelity: str = "/steps"
    secondary_stat: str = "val_ppl"
    d_model: int = 768
    member_defaults: Dict = dataclasses.field(default_factory=lambda: {"beta2": 0.95})

    def member_config(self, params: Dict, seed: int) -> MemberConfig:
        return MemberConfig(width=self.d_model, lr=float(params["/lr"]),
                            momentum=float(params.get("/beta1", 0.9)),
                            weight_decay=float(params.get("/weight_decay", 0.0)),
                            dropout=0.0, seed=int(seed) & 0x7FFFFFFF, **self.member_defaults)

    def budget(self, params: Dict) -> int:
        return int(params[self.fidelity])

    def key(self, params: Dict) -> str:
        from .mlp import param_key
        return param_key(params, self.fidelity)

    @staticmethod
    def seed_of(key: str) -> int:
        return int(key[:8], 16)
