"""Llama-style decoder LMs trained as device populations (BASELINE.json configs 4 and 5).

``PopulationLM`` keeps ``capacity`` trials of ONE architecture on a GPU.  Every parameter tensor
is stacked over the population (``[P, ...]``), so a step is a handful of batched launches
regardless of ``P``:

* GEMMs: ``pbmm`` over the population dimension -- the hand-written gfx950 population GEMM
  (``ops/gemm.py`` -> ``csrc/pgemm.hip`` ``pgemm_big_kernel``: bf16 MFMA 16x16x32, f32
  accumulation, the SwiGLU and RoPE epilogues fused); no library GEMM runs in the step;
* embedding gather/scatter, RMSNorm, RoPE + head split, causal flash attention, SwiGLU, the
  vocabulary cross-entropy and the per-trial fused AdamW: hand-written gfx950 kernels
  (:mod:`metaopt_amd.ops.lm`);
* parameters live in flat buffers -- bf16 working copy ``p16`` (autograd leaves are views of it,
  with their ``.grad`` pre-bound to views of the flat bf16 gradient ``g16``), the f32 master
  (on the GPU split: ``p16`` is its high half, ``plo`` the int16 low half), AdamW moments
  ``m``/``v`` -- so the optimizer is ONE fused kernel over all tensors and trials,
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
from typing import ClassVar, Dict, Optional

import numpy as np
import torch

from ..ops import lm as ops
from ..ops.gemm import pbmm
from ..ops.population import MemberConfig
from .flatpop import FlatPopulation

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


def _lin(x, w):
    """Population linear layer; the weight gradient goes straight into the leaf's preset
    ``.grad`` (a view of the flat gradient buffer the fused AdamW reads)."""
    return pbmm(x, w, w.grad if w.requires_grad else None)


class PopulationLM(FlatPopulation):
    """``capacity`` Llama-style LM trials of one architecture (AdamW, per-trial lr / betas /
    weight decay, per-trial gradient clipping)."""

    optimizer = "adamw"
    secondary = "ppl"

    def __init__(self, capacity: int, config="tiny-2layer", batch_size: int = 8,
                 seq_len: Optional[int] = None, device="cuda", max_grad_norm: float = 1.0,
                 eval_batch: Optional[int] = None, use_graph: bool = True,
                 moment_dtype: Optional[torch.dtype] = None):
        if moment_dtype is not None:       # AdamW first-moment storage (mopt sweep --dtype)
            self.moment_dtype = moment_dtype
        self.cfg = PRESETS[config] if isinstance(config, str) else config
        if seq_len is not None:
            self.cfg = dataclasses.replace(self.cfg, seq_len=seq_len)
        c = self.cfg
        if c.head_dim != 64 or c.seq_len % 64:
            raise ValueError("the attention kernel needs head_dim 64 and seq_len % 64 == 0")
        self.batch_size = int(batch_size)          # sequences per trial per step
        self.eval_batch = int(eval_batch or batch_size)
        self.tokens_per_step = self.batch_size * c.seq_len
        super().__init__(capacity, device=device, max_grad_norm=max_grad_norm,
                         use_graph=use_graph)
        self.cos, self.sin = ops.rope_tables(c.seq_len, c.rope_base, device=self.device)

    def param_specs(self):
        return param_specs(self.cfg)

    # AdamW first moment in bf16 (28 -> 24 bytes per parameter per step)
    moment_dtype = torch.bfloat16

    def direct_grads(self):
        # projections (pgemm grad_out), norms and the embedding (cast into the .grad views)
        return {name for name, _, _ in self.specs}

    def rows_per_batch(self, x) -> int:
        return int(x.numel())

    def train_rows(self) -> int:
        return self.tokens_per_step

    def _loss(self, tok: torch.Tensor, labels: torch.Tensor, train: bool):
        tok, labels = self._expand(tok, torch.int32), self._expand(labels, torch.int32)
        c, P = self.cfg, self.capacity
        T, d, H = c.seq_len, c.d_model, c.n_heads
        rpt = tok.numel() // P
        R = tok.numel()
        W = self.W
        x = ops.embedding(tok.reshape(-1), W["embed"], rpt)
        # every residual add is fused into the pre-norm that follows it (ops.add_rmsnorm); the
        # embedding's two gradients (residual stream, first norm) meet in that norm's backward
        x, h = ops.rmsnorm_pass(x, W["l0.attn_norm"], rpt, c.norm_eps)
        for l in range(c.n_layers):
            # interleaved-pair RoPE applied by the QKV GEMM's epilogue and, backward, by the
            # attention kernels' gradient outputs (ops.qkv_rope_attention)
            o = ops.qkv_rope_attention(h.view(P, rpt, d), W[f"l{l}.wqkv"], self.cos, self.sin,
                                       T, H)
            x, h = ops.add_rmsnorm(x, _lin(o.view(P, rpt, d), W[f"l{l}.wo"]).view(R, d),
                                   W[f"l{l}.mlp_norm"], rpt, c.norm_eps)
            # gate / up columns interleaved in 16-column groups: the SwiGLU runs in the GEMM
            # epilogues (ops.swiglu_mlp)
            y = ops.swiglu_mlp(h.view(P, rpt, d), W[f"l{l}.wgu"], W[f"l{l}.wdown"])
            nxt = W[f"l{l + 1}.attn_norm"] if l + 1 < c.n_layers else W["final_norm"]
            x, h = ops.add_rmsnorm(x, y.view(R, d), nxt, rpt, c.norm_eps)
        logits = _lin(h.view(P, rpt, d), W["head"]).view(R, c.vocab)
        if train:
            return ops.cross_entropy(logits, labels.reshape(-1), rpt, grad_scale=1.0 / rpt,
                                     unit_weights=True)
        return ops.ce_eval(logits, labels.reshape(-1), rpt)


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
    # key(params) == param_key(params, fidelity): the sweep may derive it from points directly
    key_by_params: ClassVar[bool] = True
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
