"""Unrolled-hypergradient meta-optimisation of (learning rate, momentum) on a small transformer LM
(BASELINE.json config 4).

``HypergradLM`` trains ``P`` independent inner runs of a Llama-style LM (the ``tiny-2layer``
preset by default) with SGD-momentum, and propagates forward-mode tangents of the weights with
respect to the two hyper-parameters through every inner step (Franceschi et al., "Forward and
Reverse Gradient-Based Hyperparameter Optimization", ICML 2017):

* the inner loss is written so that one forward-over-reverse pass (``torch.func.jvp`` of
  ``torch.func.grad``, vmapped over the two tangents) yields the gradient and a Hessian-vector
  product along each tangent, exactly (no finite differences): every GEMM -- the projections, the attention scores and
  values, the LM head, in the forward, the backward and the tangent propagation -- is the
  second-order-differentiable population GEMM of ``ops/pgemm_ad.py`` on the hand-written MFMA
  kernel (bf16 operands, f32 accumulation); norms, RoPE, softmax and the loss are elementwise
  fp32 ops;
* the fused update of weights, momentum and the four tangent buffers is the hand-written K11
  kernel (``mopt_hyper_sgdm``), and the final ``<grad L_val, Z>`` reductions are ``mopt_hyper_dot``;
* ``HypergradientSweep`` runs the outer loop over ranks: every rank trains its own ``P`` inner runs
  (different seeds and data shards), the per-rank mean hypergradient is averaged with ONE
  all-reduce (C2) per outer step, and the shared (log lr, logit momentum) take an Adam step;
* intra-trial data parallelism (C3, ``dp_comm``): the ranks of a DP group hold the SAME inner
  runs and each differentiates its own shard of every minibatch; the gradient and both
  Hessian-vector products are averaged with ONE all-reduce of a packed [3, P, n] buffer per
  inner step before the K11 update, so every rank takes the identical step a single process
  would take on the whole minibatch.
  Each outer step is recorded as a trial (objective = validation loss, ``gradient`` result =
  d L_val / d(lr, momentum)) in the experiment storage, the reference's gradient-result contract.
"""
from __future__ import annotations

import ctypes
import datetime
import math
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import _lib
from ..ops import lm as ops
from ..ops.pgemm_ad import matmul
from .llama import PRESETS, LMConfig, SyntheticLM, param_specs

_lib.register_signatures({
    "mopt_hyper_sgdm": ([ctypes.c_void_p] * 11 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p],
                        ctypes.c_int),
    "mopt_hyper_dot": ([ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p],
                       ctypes.c_int),
})


class _CausalSoftmax(torch.autograd.Function):
    """p = softmax(causal_mask(scale * s)) over the last dim, with analytic derivatives:
    backward gs = scale p (g - <p, g>), tangent dp = scale p (ds - <p, ds>) -- a handful of
    fused-size ops instead of the scale / masked_fill / softmax chain differentiated op by op
    (masked entries have p = 0, so no mask is needed after the forward).  The backward is
    written in differentiable ops, so forward-over-reverse (jvp of grad) composes; vmap rule
    generated."""
    generate_vmap_rule = True

    @staticmethod
    def forward(s, scale):
        T = s.shape[-1]
        mask = torch.ones(T, T, dtype=torch.bool, device=s.device).triu(1)
        return (s * scale).masked_fill(mask, float("-inf")).softmax(-1)

    @staticmethod
    def setup_context(ctx, inputs, output):
        ctx.save_for_backward(output)
        ctx.save_for_forward(output)
        ctx.scale = inputs[1]

    @staticmethod
    def backward(ctx, g):
        p, = ctx.saved_tensors
        pg = p * g
        return (pg - p * pg.sum(-1, keepdim=True)) * ctx.scale, None

    @staticmethod
    def jvp(ctx, ds, _):
        p, = ctx.saved_tensors
        pd = p * ds
        return (pd - p * pd.sum(-1, keepdim=True)) * ctx.scale


class _Rotary(torch.autograd.Function):
    """RoPE rotation of [..., T, 64] by (cos, sin) [T, 32].  The rotation is linear and
    orthogonal: its tangent is the same rotation of the input tangent and its adjoint the
    rotation by -sin, both computed by this Function again -- so every derivative order stays a
    handful of elementwise ops (no slice-gradient zero fills or cat-backward copies)."""
    generate_vmap_rule = True

    @staticmethod
    def forward(t, cos, sin):
        t1, t2 = t[..., :32], t[..., 32:]
        return torch.cat([t1 * cos - t2 * sin, t2 * cos + t1 * sin], -1)

    @staticmethod
    def setup_context(ctx, inputs, output):
        ctx.cs = (inputs[1], inputs[2])

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.cs
        return _Rotary.apply(g, cos, -sin), None, None

    @staticmethod
    def jvp(ctx, dt, _c, _s):
        cos, sin = ctx.cs
        return _Rotary.apply(dt, cos, sin)


def rope_split(qkv, cos, sin, T, H):
    """(q, k, v) [B', H, T, 64] of the fused projection rows [B' T, 3 H 64], q and k rotated
    (fp32 twin of ``ops.rope_split_ref`` with the rotation as one differentiable Function)."""
    Bp = qkv.shape[0] // T
    x = qkv.view(Bp, T, 3, H, 64).permute(2, 0, 3, 1, 4)      # [3, B', H, T, 64]
    return _Rotary.apply(x[0], cos, sin), _Rotary.apply(x[1], cos, sin), x[2].contiguous()


def rmsnorm(x, w, rows_per_trial, eps):
    """fp32 RMSNorm of rows [P rpt, d] with per-trial weights [P, d] broadcast over the trial's
    rows (``ops.rmsnorm_ref`` materialises them with repeat_interleave; same arithmetic)."""
    r = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)
    return ((x * r).view(w.shape[0], rows_per_trial, -1) * w[:, None, :]).view(x.shape)


class _SwiGLU(torch.autograd.Function):
    """silu(g) * u of gu = [g | u] with analytic derivatives (slicing gu op by op makes the
    backward zero-fill and add two full-size gradients per pass):
    adjoint [gy u silu'(g) | gy silu(g)], tangent silu'(g) u dg + silu(g) du,
    silu'(g) = s (1 + g (1 - s)), s = sigmoid(g)."""
    generate_vmap_rule = True

    @staticmethod
    def forward(gu):
        F = gu.shape[-1] // 2
        return torch.nn.functional.silu(gu[..., :F]) * gu[..., F:]

    @staticmethod
    def setup_context(ctx, inputs, output):
        ctx.save_for_backward(inputs[0])
        ctx.save_for_forward(inputs[0])

    @staticmethod
    def backward(ctx, gy):
        gu, = ctx.saved_tensors
        F = gu.shape[-1] // 2
        g, u = gu[..., :F], gu[..., F:]
        s = torch.sigmoid(g)
        return torch.cat([gy * u * (s * (1 + g * (1 - s))), gy * (g * s)], -1)

    @staticmethod
    def jvp(ctx, dgu):
        gu, = ctx.saved_tensors
        F = gu.shape[-1] // 2
        g, u = gu[..., :F], gu[..., F:]
        s = torch.sigmoid(g)
        return dgu[..., :F] * u * (s * (1 + g * (1 - s))) + (g * s) * dgu[..., F:]


def causal_attention(q, k, v, scale):
    """Causal softmax attention of [B', H, T, Dh] heads -> rows [B' T, H Dh]: scores and values
    on the population GEMM (differentiable to second order), softmax in fp32."""
    Bp, H, T, Dh = q.shape
    s = matmul(q.reshape(Bp * H, T, Dh), k.reshape(Bp * H, T, Dh), tb=True)
    p = _CausalSoftmax.apply(s, scale)
    o = matmul(p, v.reshape(Bp * H, T, Dh))
    return o.view(Bp, H, T, Dh).permute(0, 2, 1, 3).reshape(Bp * T, H * Dh)


def lm_losses(params: Dict[str, torch.Tensor], tok, tgt, cfg: LMConfig, cos, sin):
    """Per-trial mean token loss [P] of a population LM, differentiable to second order."""
    P = tok.shape[0]
    T, d, H = cfg.seq_len, cfg.d_model, cfg.n_heads
    rpt = tok[0].numel()
    R = P * rpt
    x = ops.embed_ref(tok.reshape(-1), params["embed"], rpt)
    for l in range(cfg.n_layers):
        h = rmsnorm(x, params[f"l{l}.attn_norm"], rpt, cfg.norm_eps)
        qkv = matmul(h.view(P, rpt, d), params[f"l{l}.wqkv"]).reshape(R, 3 * d)
        q, k, v = rope_split(qkv, cos, sin, T, H)
        o = causal_attention(q, k, v, 1.0 / math.sqrt(cfg.head_dim))
        x = x + matmul(o.view(P, rpt, d), params[f"l{l}.wo"]).reshape(R, d)
        h = rmsnorm(x, params[f"l{l}.mlp_norm"], rpt, cfg.norm_eps)
        a = _SwiGLU.apply(matmul(h.view(P, rpt, d), params[f"l{l}.wgu"]))
        x = x + matmul(a, params[f"l{l}.wdown"]).reshape(R, d)
    h = rmsnorm(x, params["final_norm"], rpt, cfg.norm_eps)
    logits = matmul(h.view(P, rpt, d), params["head"]).reshape(R, cfg.vocab)
    lz = torch.nn.functional.cross_entropy(logits, tgt.reshape(-1).long(), reduction="none")
    return lz.view(P, rpt).mean(1)


def hyper_sgdm_ref(w, v, ze, zm, ye, ym, g, he, hm, eta, mu):
    """fp32 reference of the K11 update (in place)."""
    e, m = eta[:, None], mu[:, None]
    vn = m * v + g
    yen = m * ye + he
    ymn = m * ym + hm + v
    ze.sub_(e * yen + vn)
    zm.sub_(e * ymn)
    w.sub_(e * vn)
    v.copy_(vn)
    ye.copy_(yen)
    ym.copy_(ymn)


class _Unflatten(torch.autograd.Function):
    """The parameter tensors of the flat run state ``W [P, n]`` (slices, reshaped).

    Differentiating through plain slices of one flat tensor makes autograd build, for EVERY
    parameter, a zero-filled [P, n] gradient holding its slice and then add them all up (and,
    forward-over-reverse, the same again for the batched tangents): ~17 full-size fills + adds
    per gradient.  Here the backward is one ``cat`` of the parameter gradients and the tangent
    of each output is the matching slice of the input tangent -- still composable with
    ``torch.func`` (jvp of the backward = cat of the tangents; vmap rule generated)."""
    generate_vmap_rule = True

    @staticmethod
    def forward(W, layout):
        return tuple(W[:, o:o + k].reshape(W.shape[0], *shape) for o, k, shape in layout)

    @staticmethod
    def setup_context(ctx, inputs, output):
        ctx.layout = inputs[1]

    @staticmethod
    def backward(ctx, *grads):
        parts = []
        for g, (o, k, shape) in zip(grads, ctx.layout):
            if g is None:
                g = torch.zeros(grads[0].shape[0], k, dtype=grads[0].dtype,
                                device=grads[0].device)
            parts.append(g.reshape(g.shape[0], k))
        return torch.cat(parts, 1), None

    @staticmethod
    def jvp(ctx, dW, _):
        return tuple(dW[:, o:o + k].reshape(dW.shape[0], *shape) for o, k, shape in ctx.layout)


class HypergradLM:
    def __init__(self, capacity: int, config="tiny-2layer", batch_size: int = 4,
                 seq_len: Optional[int] = None, device="cuda", graph: Optional[bool] = None,
                 dp_comm=None, mode: Optional[str] = None):
        cfg = PRESETS[config] if isinstance(config, str) else config
        if seq_len is not None:
            import dataclasses
            cfg = dataclasses.replace(cfg, seq_len=seq_len)
        self.cfg = cfg
        self.device = torch.device(device)
        self.P = P = int(capacity)
        self.batch_size = batch_size
        self.specs = param_specs(cfg)
        self.offsets = []
        n = 0
        for _, shape, _ in self.specs:
            k = int(np.prod(shape))
            self.offsets.append((n, k))
            n += k
        self.n = n = (n + 7) // 8 * 8
        z = lambda: torch.zeros(P, n, dtype=torch.float32, device=self.device)  # noqa: E731
        self.w, self.v, self.ye, self.ym = z(), z(), z(), z()
        # the two weight tangents are one [2, P, n] tensor (and the explicit step's gradient
        # outputs one [3, P, n]): a parameter's tangent slices are then one strided operand of
        # the two-level-batched GEMMs (models/hyper_step.py)
        self.Z = torch.zeros(2, P, n, dtype=torch.float32, device=self.device)
        self.ze, self.zm = self.Z[0], self.Z[1]
        self.eta = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.mu = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.cos, self.sin = ops.rope_tables(cfg.seq_len, cfg.rope_base, device=self.device)
        self.steps = 0
        # "explicit" (default): the hand-derived stacked forward-over-reverse step of
        # models/hyper_step.py (HIP kernels on the GPU); "func": torch.func jvp-of-grad over the
        # op-by-op graph of lm_losses (the executable specification the explicit step is tested
        # against)
        if mode is None:
            import os
            mode = os.environ.get("MOPT_HYPER_MODE", "explicit")
        if mode not in ("explicit", "func"):
            raise ValueError(f"HypergradLM: mode must be 'explicit' or 'func', got {mode!r}")
        self.mode = mode
        self._steppers = {}
        self.g = self.he = self.hm = None
        if mode == "explicit":
            self.G = torch.zeros(3, P, n, dtype=torch.float32, device=self.device)
            self.g, self.he, self.hm = self.G[0], self.G[1], self.G[2]
        # the inner step is thousands of small launches (forward, backward and two tangent
        # passes through every op): on the GPU it is captured once into a HIP graph and
        # replayed (MOPT_HYPER_GRAPH=0 runs it eagerly)
        if graph is None:
            import os
            graph = os.environ.get("MOPT_HYPER_GRAPH", "1") != "0"
        # C3: the DP group's all-reduce sits between the captured compute and the update, so
        # the step runs eagerly when the runs are data-parallel
        self.dp_comm = dp_comm if dp_comm is not None and dp_comm.world_size > 1 else None
        self.use_graph = bool(graph) and self.device.type == "cuda" and self.dp_comm is None
        self._graph = None
        self._static = None
        self._eager_steps = 0

    def params(self, W: torch.Tensor) -> Dict[str, torch.Tensor]:
        layout = tuple((o, k, tuple(shape)) for (_, shape, _), (o, k) in
                       zip(self.specs, self.offsets))
        return dict(zip((name for name, _, _ in self.specs), _Unflatten.apply(W, layout)))

    def reset(self, seeds: List[int], eta, mu) -> None:
        """Fresh inner runs: weights from per-run seeds, zero momentum and tangents."""
        for buf in (self.v, self.ze, self.zm, self.ye, self.ym):
            buf.zero_()
        self.w.zero_()
        for p, seed in enumerate(seeds):
            gen = torch.Generator(device=self.device)
            gen.manual_seed(int(seed) & 0x7FFFFFFF)
            for (name, shape, init), (o, k) in zip(self.specs, self.offsets):
                dst = self.w[p, o:o + k]
                if init[0] == "ones":
                    dst.fill_(1.0)
                else:
                    dst.normal_(0.0, init[1], generator=gen)
        self.eta.copy_(torch.as_tensor(eta, dtype=torch.float32).expand(self.P))
        self.mu.copy_(torch.as_tensor(mu, dtype=torch.float32).expand(self.P))
        self.steps = 0

    def _loss_sum(self, W, tok, tgt):
        return lm_losses(self.params(W), tok, tgt, self.cfg, self.cos, self.sin).sum()

    def _expand(self, t):
        t = t.to(self.device)
        return t.unsqueeze(0).expand(self.P, *t.shape) if t.dim() == 2 else t

    def inner_step(self, tok, tgt) -> torch.Tensor:
        """One SGD-momentum step of every run with tangent propagation; returns losses [P]."""
        tok, tgt = self._expand(tok), self._expand(tgt)
        if not self.use_graph:
            return self._step_body(tok, tgt)
        if self._graph is None and self._eager_steps < 1:
            self._eager_steps += 1            # first step eager: lazy initialisations run
            return self._step_body(tok, tgt)
        if self._graph is None:
            self._static = (tok.clone(), tgt.clone())
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._graph_out = self._step_body(*self._static)
            self.steps -= 1                    # capture recorded the step, replay runs it
        self._static[0].copy_(tok)
        self._static[1].copy_(tgt)
        self._graph.replay()
        self.steps += 1
        return self._graph_out.clone()

    def _stepper(self, S: int, B: int):
        from .hyper_step import SecondOrderStep
        key = (S, B)
        if key not in self._steppers:
            self._steppers[key] = SecondOrderStep(self.cfg, self.specs, self.offsets, self.P, B,
                                                  S, self.device, self.cos, self.sin)
        return self._steppers[key]

    def _step_body(self, tok, tgt) -> torch.Tensor:
        if self.mode == "explicit":
            losses = self._stepper(3, tok.shape[1]).run(self.w, self.Z, tok, tgt, self.G)
            g, he, hm = self.g, self.he, self.hm
        else:
            g, he, hm, losses = self._func_grads(tok, tgt)
        if self.dp_comm is not None:                                            # C3
            packed = torch.stack([g, he, hm])
            buf = packed.to(self.dp_comm._coll_device())
            self.dp_comm.all_reduce_mean_(buf)
            g, he, hm = buf.to(self.device).unbind(0)
            losses = losses.to(self.dp_comm._coll_device())
            self.dp_comm.all_reduce_mean_(losses)
            losses = losses.to(self.device)
        self._update(g.contiguous(), he.contiguous(), hm.contiguous())
        self.steps += 1
        return losses.clone() if self.mode == "explicit" else losses

    def _func_grads(self, tok, tgt):
        def loss_fn(W):
            per_trial = lm_losses(self.params(W), tok, tgt, self.cfg, self.cos, self.sin)
            return per_trial.sum(), per_trial.detach()

        grad_fn = torch.func.grad_and_value(loss_fn, has_aux=True)

        def along(tangent):
            (g, (_, losses)), (h, _) = torch.func.jvp(grad_fn, (self.w,), (tangent,))
            return g, losses, h

        # both tangents in ONE forward-over-reverse pass: vmapped over the tangent, the primal
        # forward / backward run once and every tangent op is batched (the population GEMM's
        # batching rule folds the two tangents into its trial dimension) -- half the passes of
        # one jvp per hyper-parameter, same numbers
        g, losses, h = torch.func.vmap(along, out_dims=(None, None, 0))(
            self.Z)
        return g, h[0], h[1], losses

    def _update(self, g, he, hm):
        if self.device.type == "cuda":
            lib = _lib.get_lib()
            _lib.check(lib.mopt_hyper_sgdm(*(t.data_ptr() for t in (
                self.w, self.v, self.ze, self.zm, self.ye, self.ym, g, he, hm, self.eta,
                self.mu)), self.n, self.P, _lib.stream_ptr(self.device)), "hyper_sgdm")
        else:
            hyper_sgdm_ref(self.w, self.v, self.ze, self.zm, self.ye, self.ym, g, he, hm,
                           self.eta, self.mu)

    def hypergradient(self, tok, tgt):
        """(d L_val / d eta, d L_val / d mu) per run [P, 2] and the validation losses [P]."""
        tok, tgt = self._expand(tok), self._expand(tgt)
        if self.mode == "explicit":
            gval = self.w.new_empty(1, *self.w.shape)
            losses = self._stepper(1, tok.shape[1]).run(self.w, [], tok, tgt, gval).clone()
            gval = gval[0]
        else:
            gval, lval = torch.func.grad_and_value(lambda W: self._loss_sum(W, tok, tgt))(self.w)
            with torch.no_grad():
                losses = lm_losses(self.params(self.w), tok, tgt, self.cfg, self.cos, self.sin)
        gval = gval.contiguous()
        if self.dp_comm is not None:      # C3: validation gradient over the DP group's shards
            buf = torch.cat([gval, losses[:, None]], 1).to(self.dp_comm._coll_device())
            self.dp_comm.all_reduce_mean_(buf)
            buf = buf.to(self.device)
            gval, losses = buf[:, :-1].contiguous(), buf[:, -1].contiguous()
        if self.device.type == "cuda":
            out = torch.empty(self.P, 2, dtype=torch.float32, device=self.device)
            lib = _lib.get_lib()
            _lib.check(lib.mopt_hyper_dot(gval.data_ptr(), self.ze.data_ptr(), self.zm.data_ptr(),
                                          out.data_ptr(), self.n, self.P,
                                          _lib.stream_ptr(self.device)), "hyper_dot")
        else:
            out = torch.stack([(gval * self.ze).sum(1), (gval * self.zm).sum(1)], 1)
        return out, losses


class HypergradientSweep:
    """Outer loop: shared (lr, momentum) meta-learned from ``world * P`` unrolled inner runs.

    Every outer step: rank 0 broadcasts the current hyper-parameters (C5), each rank resets its
    runs (seeds differ per rank, run and step), trains ``inner_steps`` with tangents, computes
    the hypergradient on its validation shard, and ONE all-reduce averages [d/d lr, d/d mu,
    val loss] across ranks (C2).  The meta-parameters (log lr, logit mu) then take an Adam step.
    """

    def __init__(self, model: HypergradLM, data: SyntheticLM, comm=None, experiment=None,
                 lr0: float = 0.05, mu0: float = 0.5, meta_lr: float = 0.1,
                 inner_steps: int = 20):
        from ..parallel.comm import Comm
        self.model, self.data = model, data
        self.comm = comm or Comm(device=model.device)
        self.experiment = experiment
        self.theta = np.array([math.log(lr0), math.log(mu0 / (1 - mu0))], dtype=np.float64)
        self.meta_lr = meta_lr
        self.inner_steps = inner_steps
        self._m = np.zeros(2)
        self._v = np.zeros(2)
        self.history: List[dict] = []
        self.outer = 0

    @property
    def hparams(self):
        return float(math.exp(self.theta[0])), float(1 / (1 + math.exp(-self.theta[1])))

    def step(self) -> dict:
        comm, model = self.comm, self.model
        theta = torch.tensor(self.theta, dtype=torch.float64, device=comm._coll_device())
        comm.broadcast_(theta, src=0)                                           # C5
        self.theta = theta.cpu().numpy()
        lr, mu = self.hparams
        dp = model.dp_comm is not None
        if dp:   # C3: the same runs on every rank, each rank differentiating its rows
            base, shard = self.outer * model.P, self.outer
        else:
            base = (self.outer * comm.world_size + comm.rank) * model.P
            shard = self.outer * comm.world_size + comm.rank
        model.reset([1000003 * (base + p) + 17 for p in range(model.P)], lr, mu)
        for k in range(self.inner_steps):
            tok, tgt = self.data.batch(shard * self.inner_steps + k)
            if dp:
                if tok.shape[0] % comm.world_size:
                    raise ValueError(f"C3: the minibatch ({tok.shape[0]} rows) does not split "
                                     f"evenly over {comm.world_size} ranks; the averaged "
                                     "shard gradients would not equal the full batch's")
                rows = tok.shape[0] // comm.world_size
                tok = tok[comm.rank * rows:(comm.rank + 1) * rows]
                tgt = tgt[comm.rank * rows:(comm.rank + 1) * rows]
            model.inner_step(tok, tgt)
        hg, vl = model.hypergradient(*self.data.validation())
        red = torch.cat([hg.mean(0).double(), vl.mean().double().view(1)])
        red = red.to(comm._coll_device())
        comm.all_reduce_mean_(red)                                              # C2
        g_lr, g_mu, val = (float(x) for x in red.cpu())
        # chain rule into the unconstrained meta-parameters, then Adam
        grad = np.array([g_lr * lr, g_mu * mu * (1 - mu)])
        self.outer += 1
        b1, b2 = 0.9, 0.999
        self._m = b1 * self._m + (1 - b1) * grad
        self._v = b2 * self._v + (1 - b2) * grad ** 2
        mh = self._m / (1 - b1 ** self.outer)
        vh = self._v / (1 - b2 ** self.outer)
        self.theta = self.theta - self.meta_lr * mh / (np.sqrt(vh) + 1e-8)
        rec = {"outer": self.outer, "lr": lr, "momentum": mu, "val_loss": val,
               "d_lr": g_lr, "d_momentum": g_mu}
        self.history.append(rec)
        if comm.is_root and self.experiment is not None:
            self._record(rec)
        return rec

    def _record(self, rec):
        from ..core.trial import Trial
        exp = self.experiment
        now = datetime.datetime.utcnow()
        t = Trial(experiment=exp.id, status="completed",
                  params=[dict(name="/lr", type="real", value=rec["lr"]),
                          dict(name="/momentum", type="real", value=rec["momentum"])],
                  results=[dict(name="val_loss", type="objective", value=rec["val_loss"]),
                           dict(name="hypergradient", type="gradient",
                                value=[rec["d_lr"], rec["d_momentum"]])])
        t.submit_time = t.start_time = t.end_time = now
        try:
            exp.storage.register_trial(t)
        except Exception:  # duplicate point (same lr/mu twice): keep the first record
            pass

    def run(self, outer_steps: int) -> List[dict]:
        for _ in range(outer_steps):
            self.step()
        return self.history
