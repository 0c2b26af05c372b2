"""Hand-derived forward-over-reverse inner step of the unrolled hypergradient (K11, config 4).

``SecondOrderStep`` computes, for every run of a population LM (``models/llama.py`` layout,
parameters in the flat ``[P, n]`` state of ``HypergradLM``), the training-loss gradient ``g``
AND its directional derivatives ``H Z_t`` along the weight tangents ``Z_t`` (one per
hyper-parameter), without ``torch.func``: every activation is carried as a STACK of ``S``
slices -- slice 0 the primal value, slices 1..S-1 its tangents -- stored ``[P, S * rows, cols]``
(each trial's slices are consecutive row blocks), and every operator has a forward that maps
stacks to stacks and a backward that maps (primal + tangent) adjoints back.  With ``S = 1`` the
same code is a plain forward/backward (the validation gradient of ``hypergradient()``).

Per operator (primal ``y = f(x, w)``, tangent ``ẏ``, adjoint ``gx``, tangent of the adjoint
``ġx``):

* linear ``y = x W``: ``ẏ = ẋ W + x Ẇ``; ``gx = gy Wᵀ``, ``ġx = ġy Wᵀ + gy Ẇᵀ``;
  ``G = xᵀ gy``, ``Ġ = ẋᵀ gy + xᵀ ġy`` -- all on the population MFMA GEMM (``ops/gemm.py``,
  f32 activations rounded to bf16 while staged, f32 accumulation), the stacked slices of ``x``
  and ``gy`` as extra rows of one GEMM, the ``Ẇ`` terms accumulated into their slices by the
  GEMM epilogue (``res``), the residual adds of the transformer blocks folded in the same way;
* RMSNorm ``y = n a``, ``n = x r``, ``r = (mean x² + eps)^-1/2``:
  ``ṅ = r (ẋ - n <n, ẋ>/d)``; ``gx = r (gn - n c)``, ``c = <n, gn>/d``, ``gn = gy a``;
  ``ġx = ṙ (gn - n c) + r (ġn - ṅ c - n ċ)`` with ``ṙ = -r² <n, ẋ>/d``,
  ``ċ = (<ṅ, gn> + <n, ġn>)/d``, ``ġn = ġy a + gy ȧ``;  ``Ga = Σ gy n``, ``Ġa = Σ ġy n + gy ṅ``;
* RoPE: linear and orthogonal, the same rotation of every slice; adjoint = rotation by ``-sin``;
* causal attention ``o = P v``, ``P = softmax(scale q kᵀ)`` on the materialised per-head
  ``T x T`` score tiles (GEMMs on MFMA, the softmax and its derivatives in one fused kernel each
  way): ``Ṗ = P ∘ (ṡ - <P, ṡ>)``, ``ȯ = Ṗ v + P v̇``;  ``gs = P ∘ (gP - D)``,
  ``ġs = Ṗ ∘ (gP - D) + P ∘ (ġP - Ḋ)`` with ``D = <go, o>``, ``Ḋ = <ġo, o> + <go, ȯ>``;
* SwiGLU ``y = silu(g) u``: ``ẏ = silu'(g) ġ u + silu(g) u̇``; ``gg = gy u silu'(g)``,
  ``gu = gy silu(g)``, ``ġg = (ġy u + gy u̇) silu'(g) + gy u silu''(g) ġ``,
  ``ġu = ġy silu(g) + gy silu'(g) ġ``;
* token cross-entropy (mean over a trial's rows): ``gz = (π - onehot)/R``,
  ``ġz = π ∘ (ż - <π, ż>)/R``;
* embedding: a gather of the table and of its tangents; adjoint = scatter-add of each slice.

``TorchStackOps`` is the fp32 PyTorch definition of every stacked operator (the CPU path and
the numerics reference of the tests, which also pin it against ``torch.func`` on the op-by-op
graph of ``models/hyper.lm_losses``); ``HipStackOps`` runs the same operators as the HIP
kernels of ``ops/csrc/hyper_kernels.hip``.  On the GPU the whole step is a fixed launch
sequence, captured once into a HIP graph by ``HypergradLM``.
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Optional, Sequence

import torch

from ..ops import _lib
from ..ops.gemm import pgemm

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float

_lib.register_signatures({
    "mopt_hy_embed_fwd": ([_P, _L, _P, _P, _P, _P, _I, _I, _I, _I, _L, _P], _I),
    "mopt_hy_embed_bwd": ([_P, _L, _P, _P, _P, _P, _I, _I, _I, _I, _L, _P], _I),
    "mopt_hy_norm_fwd": ([_P] * 6 + [_I] * 4 + [_L, _F, _P], _I),
    "mopt_hy_norm_bwd": ([_P] * 10 + [_I] * 4 + [_L, _I, _P], _I),
    "mopt_hy_rope": ([_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P], _I),
    "mopt_hy_heads": ([_P, _P, _I, _I, _I, _I, _I, _I, _P], _I),
    "mopt_hy_softmax_fwd": ([_P, _P, _P, _I, _I, _I, _F, _P], _I),
    "mopt_hy_softmax_bwd": ([_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P], _I),
    "mopt_hy_swiglu": ([_P, _P, _P, _I, _I, _I, _I, _P], _I),
    "mopt_hy_ce": ([_P, _P, _L, _P, _I, _I, _I, _I, _P], _I),
    "mopt_hy_zero": ([_P, _P, _P, _I, _L, _P, _P, _I, _P], _I),
})


# ============================================================================ stacked operators
class TorchStackOps:
    """fp32 PyTorch definition of the stacked operators (``S`` slices, slice 0 = primal).
    Shapes: ``X [P, S*R, d]`` (trial p's slices are its consecutive row blocks)."""

    def __init__(self, S: int):
        self.S = S

    # ------------------------------------------------------------------ embedding
    def embed_fwd(self, tok, E: Sequence[torch.Tensor], out):
        """out[:, s*R + r] = E_s[p, tok[p, r]] (E_0 the table, E_1.. its tangents)."""
        P, R = tok.shape
        pidx = torch.arange(P, device=tok.device)[:, None]
        for s in range(self.S):
            out[:, s * R:(s + 1) * R] = E[s][pidx, tok.long()]

    def embed_bwd(self, tok, GX, G: Sequence[torch.Tensor]):
        """G_s[p, tok[p, r]] += GX[p, s*R + r] (G_s zero-filled by the caller)."""
        P, R = tok.shape
        for s in range(self.S):
            for p in range(P):
                G[s][p].index_add_(0, tok[p].long(), GX[p, s * R:(s + 1) * R])

    # ------------------------------------------------------------------ RMSNorm
    def norm_fwd(self, X, a: Sequence[torch.Tensor], Y, rstd, eps):
        R = X.shape[1] // self.S
        x = X[:, :R]
        r = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)
        n = x * r
        Y[:, :R] = n * a[0][:, None, :]
        rstd.copy_(r[..., 0])
        for t in range(1, self.S):
            xd = X[:, t * R:(t + 1) * R]
            nd = r * (xd - n * (n * xd).mean(-1, keepdim=True))
            Y[:, t * R:(t + 1) * R] = nd * a[0][:, None, :] + n * a[t][:, None, :]

    def norm_bwd(self, X, GY, a, rstd, GX, G, accumulate: bool):
        """GX (+)= the input adjoint stack; G_s = the weight gradient and its tangents."""
        R = X.shape[1] // self.S
        d = X.shape[2]
        x = X[:, :R]
        r = rstd[..., None]
        n = x * r
        gy = GY[:, :R]
        gn = gy * a[0][:, None, :]
        c = (n * gn).sum(-1, keepdim=True) / d
        out = [r * (gn - n * c)]
        G[0].copy_((gy * n).sum(1))
        for t in range(1, self.S):
            xd, gyd = X[:, t * R:(t + 1) * R], GY[:, t * R:(t + 1) * R]
            cx = (n * xd).sum(-1, keepdim=True) / d
            rd = -r * r * cx
            nd = r * (xd - n * cx)
            gnd = gyd * a[0][:, None, :] + gy * a[t][:, None, :]
            cd = ((nd * gn).sum(-1, keepdim=True) + (n * gnd).sum(-1, keepdim=True)) / d
            out.append(rd * (gn - n * c) + r * (gnd - nd * c - n * cd))
            G[t].copy_((gyd * n + gy * nd).sum(1))
        res = torch.cat(out, 1)
        if accumulate:
            GX.add_(res)
        else:
            GX.copy_(res)

    # ------------------------------------------------------------------ RoPE + head split
    @staticmethod
    def _rot(t, cos, sin):
        t1, t2 = t[..., :32], t[..., 32:]
        return torch.cat([t1 * cos - t2 * sin, t2 * cos + t1 * sin], -1)

    def rope_split(self, QKV, cos, sin, B, T, H, Qh, Kh, Vh):
        """QKV [P, S*R, 3 d] (cols: q | k | v, head-major) -> Qh/Kh/Vh [P*B*H, S*T, 64],
        q and k rotated."""
        P, S = QKV.shape[0], self.S
        x = QKV.view(P, S, B, T, 3, H, 64).permute(4, 0, 2, 5, 1, 3, 6)   # [3,P,B,H,S,T,64]
        Qh.copy_(self._rot(x[0], cos, sin).reshape(Qh.shape))
        Kh.copy_(self._rot(x[1], cos, sin).reshape(Kh.shape))
        Vh.copy_(x[2].reshape(Vh.shape))

    def rope_merge(self, GQh, GKh, GVh, cos, sin, B, T, H, GQKV):
        """Adjoint of rope_split: head stacks -> GQKV [P, S*R, 3 d], q/k rotated by -sin."""
        P, S = GQKV.shape[0], self.S
        sh = (P, B, H, S, T, 64)
        parts = [self._rot(GQh.view(sh), cos, -sin), self._rot(GKh.view(sh), cos, -sin),
                 GVh.view(sh)]
        x = torch.stack(parts, 0)                                           # [3,P,B,H,S,T,64]
        GQKV.view(P, S, B, T, 3, H, 64).copy_(x.permute(1, 4, 2, 5, 0, 3, 6))

    def heads_merge(self, Oh, B, T, H, O):
        """Oh [P*B*H, S*T, 64] -> O [P, S*R, H*64]."""
        P, S = O.shape[0], self.S
        O.view(P, S, B, T, H, 64).copy_(Oh.view(P, B, H, S, T, 64).permute(0, 3, 1, 4, 2, 5))

    def heads_split(self, O, B, T, H, Oh):
        P, S = O.shape[0], self.S
        Oh.view(P, B, H, S, T, 64).copy_(O.view(P, S, B, T, H, 64).permute(0, 2, 4, 1, 3, 5))

    # ------------------------------------------------------------------ causal softmax
    def softmax_fwd(self, S1, S2, scale, Pm):
        """S1 [N, S*T, T] = Q k0ᵀ, S2 [N, T, (S-1) T] = q0 k_tᵀ  ->  Pm = [P; Ṗ_1; ...]."""
        T = S1.shape[2]
        mask = torch.ones(T, T, dtype=torch.bool, device=S1.device).triu(1)
        p = (S1[:, :T] * scale).masked_fill(mask, float("-inf")).softmax(-1)
        Pm[:, :T] = p
        for t in range(1, self.S):
            sd = scale * (S1[:, t * T:(t + 1) * T] + S2[:, :, (t - 1) * T:t * T])
            sd = sd.masked_fill(mask, 0.0)
            Pm[:, t * T:(t + 1) * T] = p * (sd - (p * sd).sum(-1, keepdim=True))

    def softmax_bwd(self, Pm, GP1, GP2, Oh, GOh, scale, GS):
        """GP1 [N, S*T, T] = GO v0ᵀ, GP2 [N, T, (S-1) T] = go0 v_tᵀ -> GS (scaled score
        adjoints [gs; ġs_1; ...])."""
        T = Pm.shape[2]
        p, gp = Pm[:, :T], GP1[:, :T]
        o, go = Oh[:, :T], GOh[:, :T]
        D = (go * o).sum(-1, keepdim=True)
        GS[:, :T] = scale * p * (gp - D)
        for t in range(1, self.S):
            sl = slice(t * T, (t + 1) * T)
            pd = Pm[:, sl]
            gpd = GP1[:, sl] + GP2[:, :, (t - 1) * T:t * T]
            Dd = (GOh[:, sl] * o).sum(-1, keepdim=True) + (go * Oh[:, sl]).sum(-1, keepdim=True)
            GS[:, sl] = scale * (pd * (gp - D) + p * (gpd - Dd))

    # ------------------------------------------------------------------ SwiGLU
    def swiglu_fwd(self, GU, A):
        R = GU.shape[1] // self.S
        F = GU.shape[2] // 2
        g, u = GU[:, :R, :F], GU[:, :R, F:]
        s = torch.sigmoid(g)
        A[:, :R] = g * s * u
        d1 = s * (1 + g * (1 - s))
        for t in range(1, self.S):
            gd, ud = GU[:, t * R:(t + 1) * R, :F], GU[:, t * R:(t + 1) * R, F:]
            A[:, t * R:(t + 1) * R] = d1 * gd * u + g * s * ud

    def swiglu_bwd(self, GU, GA, GGU):
        R = GU.shape[1] // self.S
        F = GU.shape[2] // 2
        g, u = GU[:, :R, :F], GU[:, :R, F:]
        s = torch.sigmoid(g)
        f0, d1 = g * s, s * (1 + g * (1 - s))
        d2 = s * (1 - s) * (2 + g * (1 - 2 * s))
        ga = GA[:, :R]
        GGU[:, :R, :F] = ga * u * d1
        GGU[:, :R, F:] = ga * f0
        for t in range(1, self.S):
            sl = slice(t * R, (t + 1) * R)
            gd, ud, gad = GU[:, sl, :F], GU[:, sl, F:], GA[:, sl]
            GGU[:, sl, :F] = (gad * u + ga * ud) * d1 + ga * u * d2 * gd
            GGU[:, sl, F:] = gad * f0 + ga * d1 * gd

    # ------------------------------------------------------------------ cross-entropy
    def ce(self, Z, tgt, losses):
        """In place: Z [P, S*R, V] logits stack -> adjoint stack; losses [P] = mean loss."""
        P, R = tgt.shape
        z = Z[:, :R]
        lp = torch.log_softmax(z, -1)
        pi = lp.exp()
        nll = -lp.gather(-1, tgt.long()[..., None])[..., 0]
        losses.copy_(nll.mean(1))
        for t in range(1, self.S):
            zd = Z[:, t * R:(t + 1) * R]
            Z[:, t * R:(t + 1) * R] = pi * (zd - (pi * zd).sum(-1, keepdim=True)) / R
        gz = pi.clone()
        gz.scatter_add_(-1, tgt.long()[..., None],
                        torch.full_like(gz[..., :1], -1.0))
        Z[:, :R] = gz / R

    def zero(self, bufs: Sequence[torch.Tensor], segs, losses):
        for b in bufs:
            for o, k in segs:
                b[:, o:o + k].zero_()
        if losses is not None:
            losses.zero_()


class HipStackOps(TorchStackOps):
    """The stacked operators as the HIP kernels of ``csrc/hyper_kernels.hip`` (f32 in HBM, one
    launch per operator and stack; the caller checks shapes once per step layout)."""

    def __init__(self, S: int, device):
        super().__init__(S)
        self.lib = _lib.get_lib()
        self.device = device

    def _st(self):
        return _lib.stream_ptr(self.device)

    def embed_fwd(self, tok, E, out):
        P, R = tok.shape
        d = out.shape[2]
        V = E[0].shape[1]
        e = [t.data_ptr() for t in E] + [0] * (3 - len(E))
        _lib.check(self.lib.mopt_hy_embed_fwd(tok.data_ptr(), tok.stride(0), *e, out.data_ptr(),
                                              P, R, d, V, E[0].stride(0), self._st()),
                   "hy_embed_fwd")

    def embed_bwd(self, tok, GX, G):
        P, R = tok.shape
        d = GX.shape[2]
        V = G[0].shape[1]
        gp = [t.data_ptr() for t in G] + [0] * (3 - len(G))
        _lib.check(self.lib.mopt_hy_embed_bwd(tok.data_ptr(), tok.stride(0), GX.data_ptr(), *gp,
                                              P, R, d, V, G[0].stride(0), self._st()),
                   "hy_embed_bwd")

    def norm_fwd(self, X, a, Y, rstd, eps):
        P, SR, d = X.shape
        ap = [t.data_ptr() for t in a] + [0] * (3 - len(a))
        _lib.check(self.lib.mopt_hy_norm_fwd(X.data_ptr(), *ap, Y.data_ptr(), rstd.data_ptr(),
                                             P, SR // self.S, d, self.S, a[0].stride(0),
                                             float(eps), self._st()), "hy_norm_fwd")

    def norm_bwd(self, X, GY, a, rstd, GX, G, accumulate):
        P, SR, d = X.shape
        ap = [t.data_ptr() for t in a] + [0] * (3 - len(a))
        gp = [t.data_ptr() for t in G] + [0] * (3 - len(G))
        _lib.check(self.lib.mopt_hy_norm_bwd(X.data_ptr(), GY.data_ptr(), *ap, rstd.data_ptr(),
                                             GX.data_ptr(), *gp, P, SR // self.S, d, self.S,
                                             a[0].stride(0), int(accumulate), self._st()),
                   "hy_norm_bwd")

    def rope_split(self, QKV, cos, sin, B, T, H, Qh, Kh, Vh):
        P = QKV.shape[0]
        _lib.check(self.lib.mopt_hy_rope(QKV.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                         Qh.data_ptr(), Kh.data_ptr(), Vh.data_ptr(), P, B, T, H,
                                         self.S, 0, self._st()), "hy_rope")

    def rope_merge(self, GQh, GKh, GVh, cos, sin, B, T, H, GQKV):
        P = GQKV.shape[0]
        _lib.check(self.lib.mopt_hy_rope(GQKV.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                         GQh.data_ptr(), GKh.data_ptr(), GVh.data_ptr(), P, B, T,
                                         H, self.S, 1, self._st()), "hy_rope")

    def heads_merge(self, Oh, B, T, H, O):
        _lib.check(self.lib.mopt_hy_heads(O.data_ptr(), Oh.data_ptr(), O.shape[0], B, T, H,
                                          self.S, 1, self._st()), "hy_heads")

    def heads_split(self, O, B, T, H, Oh):
        _lib.check(self.lib.mopt_hy_heads(O.data_ptr(), Oh.data_ptr(), O.shape[0], B, T, H,
                                          self.S, 0, self._st()), "hy_heads")

    def softmax_fwd(self, S1, S2, scale, Pm):
        N, _, T = S1.shape
        _lib.check(self.lib.mopt_hy_softmax_fwd(S1.data_ptr(), 0 if S2 is None else
                                                S2.data_ptr(), Pm.data_ptr(), N, T, self.S,
                                                float(scale), self._st()), "hy_softmax_fwd")

    def softmax_bwd(self, Pm, GP1, GP2, Oh, GOh, scale, GS):
        N, _, T = Pm.shape
        _lib.check(self.lib.mopt_hy_softmax_bwd(Pm.data_ptr(), GP1.data_ptr(),
                                                0 if GP2 is None else GP2.data_ptr(),
                                                Oh.data_ptr(), GOh.data_ptr(), GS.data_ptr(),
                                                N, T, self.S, float(scale), self._st()),
                   "hy_softmax_bwd")

    def swiglu_fwd(self, GU, A):
        P, SR, F2 = GU.shape
        _lib.check(self.lib.mopt_hy_swiglu(GU.data_ptr(), A.data_ptr(), 0, P, SR // self.S,
                                           F2 // 2, self.S, self._st()), "hy_swiglu")

    def swiglu_bwd(self, GU, GA, GGU):
        P, SR, F2 = GU.shape
        _lib.check(self.lib.mopt_hy_swiglu(GU.data_ptr(), GA.data_ptr(), GGU.data_ptr(), P,
                                           SR // self.S, F2 // 2, self.S, self._st()),
                   "hy_swiglu")

    def ce(self, Z, tgt, losses):
        P, R = tgt.shape
        _lib.check(self.lib.mopt_hy_ce(Z.data_ptr(), tgt.data_ptr(), tgt.stride(0),
                                       losses.data_ptr(), P, R, Z.shape[2], self.S, self._st()),
                   "hy_ce")

    def zero(self, bufs, segs, losses):
        # host arrays: the launcher copies them into the kernel's by-value arguments
        offs = (ctypes.c_int64 * len(segs))(*[o for o, _ in segs])
        lens = (ctypes.c_int64 * len(segs))(*[k for _, k in segs])
        bp = [b.data_ptr() for b in bufs] + [0] * (3 - len(bufs))
        _lib.check(self.lib.mopt_hy_zero(*bp, bufs[0].shape[0], bufs[0].stride(0),
                                         ctypes.addressof(offs), ctypes.addressof(lens),
                                         len(segs), self._st()), "hy_zero")
        if losses is not None:
            losses.zero_()


# ============================================================================ the step
class SecondOrderStep:
    """Gradient (slice 0) and tangent gradients (slices 1..S-1) of the summed per-trial mean
    token loss of a population LM, for the flat state layout of ``HypergradLM``.

    ``run(W, Z, tok, tgt, G)``: ``W [P, n]`` weights, ``Z`` the ``S-1`` weight tangents
    ``[P, n]``, ``tok``/``tgt`` ``[P, B, T]`` (any trial stride, 0 = shared batch),
    ``G`` the ``S`` output buffers ``[P, n]`` (gradient, then ``H Z_t``).  Returns the
    per-trial losses ``[P]``."""

    def __init__(self, cfg, specs, offsets, P: int, B: int, S: int, device, cos, sin,
                 backend: Optional[str] = None):
        self.cfg, self.P, self.B, self.S = cfg, P, B, S
        self.T = cfg.seq_len
        self.device = torch.device(device)
        self.cos, self.sin = cos, sin
        if backend is None:
            backend = "hip" if self.device.type == "cuda" else "torch"
        if backend == "hip" and self.device.type != "cuda":
            raise ValueError("SecondOrderStep: the hip backend needs a cuda device")
        self.backend = backend
        self.ops = HipStackOps(S, self.device) if backend == "hip" else TorchStackOps(S)
        self.layout = {name: (o, k, tuple(shape)) for (name, shape, _), (o, k)
                       in zip(specs, offsets)}
        # the embedding and norm-weight gradient slices are accumulated (scatter-add, row
        # sums): zeroed at the start of every step
        self.acc_segs = [(o, k) for name, (o, k, shape) in self.layout.items()
                         if name == "embed" or len(shape) == 1]
        if cfg.head_dim != 64:
            raise ValueError("SecondOrderStep: head_dim must be 64")
        for name, (o, k, shape) in self.layout.items():
            if o % 4 or (len(shape) == 2 and shape[1] % 8):
                raise ValueError(f"SecondOrderStep: parameter {name} is not 16-byte aligned "
                                 "for the GEMM operands")
        self._alloc()

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        c, P, B, S, T = self.cfg, self.P, self.B, self.S, self.T
        R = B * T
        d, F, V, L, H = c.d_model, c.ffn, c.vocab, c.n_layers, c.n_heads
        N = P * B * H
        f = dict(dtype=torch.float32, device=self.device)
        e = torch.empty
        self.R, self.N = R, N
        self.xs = [e(P, S * R, d, **f) for _ in range(2 * L + 1)]
        self.h1 = [e(P, S * R, d, **f) for _ in range(L)]
        self.h2 = [e(P, S * R, d, **f) for _ in range(L)]
        self.r1 = [e(P, R, **f) for _ in range(L)]
        self.r2 = [e(P, R, **f) for _ in range(L)]
        self.qkv = e(P, S * R, 3 * d, **f)
        self.Qh = [e(N, S * T, 64, **f) for _ in range(L)]
        self.Kh = [e(N, S * T, 64, **f) for _ in range(L)]
        self.Vh = [e(N, S * T, 64, **f) for _ in range(L)]
        self.Pm = [e(N, S * T, T, **f) for _ in range(L)]
        self.Oh = [e(N, S * T, 64, **f) for _ in range(L)]
        self.o = [e(P, S * R, d, **f) for _ in range(L)]
        self.gu = [e(P, S * R, 2 * F, **f) for _ in range(L)]
        self.a = [e(P, S * R, F, **f) for _ in range(L)]
        self.hf = e(P, S * R, d, **f)
        self.rf = e(P, R, **f)
        self.logits = e(P, S * R, V, **f)
        self.losses = e(P, **f)
        # scratch of the attention and the backward
        self.S1 = e(N, S * T, T, **f)
        self.S2 = e(N, T, (S - 1) * T, **f) if S > 1 else None
        self.GP2 = e(N, T, (S - 1) * T, **f) if S > 1 else None
        self.GS = e(N, S * T, T, **f)
        self.GOh = e(N, S * T, 64, **f)
        self.GQh = e(N, S * T, 64, **f)
        self.GKh = e(N, S * T, 64, **f)
        self.GVh = e(N, S * T, 64, **f)
        self.gx = e(P, S * R, d, **f)
        self.gh = e(P, S * R, d, **f)
        self.gqkv = e(P, S * R, 3 * d, **f)
        self.ga = e(P, S * R, F, **f)
        self.ggu = e(P, S * R, 2 * F, **f)
        self.go = e(P, S * R, d, **f)

    # ------------------------------------------------------------------ helpers
    # Parameters: W [P, n]; the tangents Z [S-1, P, n] and the outputs G [S, P, n] are ONE
    # tensor each, so a parameter's tangent / gradient slices form a 4-D view [P, S', K, N]
    # (dim 1 strided by P n) that one two-level-batched GEMM covers.
    def _pw(self, name):
        o, k, shape = self.layout[name]
        v = self._W[:, o:o + k]
        return v.view(self.P, *shape) if len(shape) == 2 else v

    def _p4(self, buf, name):
        """[P, S', K, N] view of parameter ``name`` in a stacked [S', P, n] buffer."""
        o, k, shape = self.layout[name]
        return buf[:, :, o:o + k].reshape(buf.shape[0], self.P, *shape).permute(1, 0, 2, 3)

    def _plist(self, name, grads=False):
        """[primal, tangent_1, ...] (or the gradient slices) of a 1-D/2-D parameter."""
        o, k, shape = self.layout[name]
        bufs = list(self._G) if grads else [self._W] + list(self._Z)
        out = [b[:, o:o + k] for b in bufs]
        return [v.view(self.P, *shape) for v in out] if len(shape) == 2 else out

    def _s4(self, X):
        """[P, S, rows, cols] view of a stack [P, S rows, cols]."""
        return X.view(X.shape[0], self.S, X.shape[1] // self.S, X.shape[2])

    def _lin_fwd(self, X, name, Y, res=None):
        """Y = X W (+ res) over every slice, then slice t += x0 Ẇ_t (one two-level GEMM)."""
        pgemm(X, self._pw(name), out=Y, res=res)
        if self.S > 1:
            x4, y4 = self._s4(X), self._s4(Y)[:, 1:]
            pgemm(x4[:, :1].expand(-1, self.S - 1, -1, -1), self._p4(self._Z, name), out=y4,
                  res=y4)

    def _linear_bwd(self, name, X, GY, GX):
        S = self.S
        x4, g4 = self._s4(X), self._s4(GY)
        G4 = self._p4(self._G, name)
        # G_s = x_sᵀ gy0 for every slice (G, then ẋ_tᵀ gy0), then Ġ_t += x0ᵀ ġy_t
        pgemm(x4, g4[:, :1].expand(-1, S, -1, -1), ta=True, out=G4)
        if S > 1:
            gt = G4[:, 1:]
            pgemm(x4[:, :1].expand(-1, S - 1, -1, -1), g4[:, 1:], ta=True, out=gt, res=gt)
        if GX is not None:
            pgemm(GY, self._pw(name), tb=True, out=GX)
            if S > 1:
                xt = self._s4(GX)[:, 1:]
                pgemm(g4[:, :1].expand(-1, S - 1, -1, -1), self._p4(self._Z, name), tb=True,
                      out=xt, res=xt)

    def _attn_fwd(self, l, scale):
        S, T = self.S, self.T
        Qh, Kh, Vh, Pm, Oh = self.Qh[l], self.Kh[l], self.Vh[l], self.Pm[l], self.Oh[l]
        pgemm(Qh, Kh[:, :T], tb=True, out=self.S1)
        if S > 1:
            pgemm(Qh[:, :T], Kh[:, T:], tb=True, out=self.S2)
        self.ops.softmax_fwd(self.S1, self.S2, scale, Pm)
        pgemm(Pm, Vh[:, :T], out=Oh)
        if S > 1:                                        # ȯ_t += P v_t
            ot = self._s4(Oh)[:, 1:]
            pgemm(self._s4(Pm)[:, :1].expand(-1, S - 1, -1, -1), self._s4(Vh)[:, 1:], out=ot,
                  res=ot)

    def _attn_bwd(self, l, scale):
        S, T = self.S, self.T
        Qh, Kh, Vh, Pm, Oh = self.Qh[l], self.Kh[l], self.Vh[l], self.Pm[l], self.Oh[l]
        GOh, GS = self.GOh, self.GS
        GP1 = self.S1                                    # scratch reuse: [N, S T, T]
        pgemm(GOh, Vh[:, :T], tb=True, out=GP1)
        if S > 1:
            pgemm(GOh[:, :T], Vh[:, T:], tb=True, out=self.GP2)
        self.ops.softmax_bwd(Pm, GP1, self.GP2, Oh, GOh, scale, GS)
        gs4, q4, k4, p4, go4 = (self._s4(t) for t in (GS, Qh, Kh, Pm, GOh))
        gq4, gk4, gv4 = (self._s4(t) for t in (self.GQh, self.GKh, self.GVh))
        b0 = lambda x, n: x[:, :1].expand(-1, n, -1, -1)        # noqa: E731
        # q: [gs; ġs_t] k0 (then ġq_t += gs k_t); k: gs_sᵀ q0 (then ġk_t += gsᵀ q_t);
        # v: P_sᵀ go0 (then ġv_t += Pᵀ ġo_t)
        pgemm(GS, Kh[:, :T], out=self.GQh)
        pgemm(gs4, b0(q4, S), ta=True, out=gk4)
        pgemm(p4, b0(go4, S), ta=True, out=gv4)
        if S > 1:
            gq, gk, gv = gq4[:, 1:], gk4[:, 1:], gv4[:, 1:]
            pgemm(b0(gs4, S - 1), k4[:, 1:], out=gq, res=gq)
            pgemm(b0(gs4, S - 1), q4[:, 1:], ta=True, out=gk, res=gk)
            pgemm(b0(p4, S - 1), go4[:, 1:], ta=True, out=gv, res=gv)

    # ------------------------------------------------------------------ the step
    def run(self, W: torch.Tensor, Z, tok, tgt, G):
        """``Z``: ``[S-1, P, n]`` tensor (or list of ``[P, n]``), ``G``: ``[S, P, n]`` tensor
        (or list; lists are staged through stacked copies)."""
        c, S, B, T, R = self.cfg, self.S, self.B, self.T, self.R
        L, H, ops = c.n_layers, c.n_heads, self.ops
        P = self.P
        Zs = Z if isinstance(Z, torch.Tensor) else (
            torch.stack(list(Z)) if len(Z) else W.new_empty(0, *W.shape))
        Gl = None
        if isinstance(G, torch.Tensor):
            Gs = G
        else:
            Gl = list(G)
            Gs = W.new_empty(len(Gl), *W.shape)
        if Zs.shape != (S - 1, *W.shape) or Gs.shape != (S, *W.shape):
            raise ValueError("SecondOrderStep: expected Z [S-1, P, n] and G [S, P, n]")
        for t in (W, Zs, Gs):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("SecondOrderStep: weights, tangents and gradient buffers must "
                                 "be contiguous f32 tensors of one layout")
        self._W, self._Z, self._G = W, Zs, Gs
        if self.backend == "hip" and (tok.dtype != torch.int32 or tgt.dtype != torch.int32):
            tok, tgt = tok.to(torch.int32), tgt.to(torch.int32)
        tok = tok.reshape(P, R) if tok.stride(0) != 0 else tok[:1].reshape(1, R).expand(P, R)
        tgt = tgt.reshape(P, R) if tgt.stride(0) != 0 else tgt[:1].reshape(1, R).expand(P, R)
        scale = 1.0 / math.sqrt(c.head_dim)
        pw = self._plist
        pg = lambda name: self._plist(name, grads=True)          # noqa: E731
        ops.zero(list(Gs), self.acc_segs, None)
        # ---------------- forward (primal + tangents)
        ops.embed_fwd(tok, pw("embed"), self.xs[0])
        for l in range(L):
            x_in, x_mid, x_out = self.xs[2 * l], self.xs[2 * l + 1], self.xs[2 * l + 2]
            ops.norm_fwd(x_in, pw(f"l{l}.attn_norm"), self.h1[l], self.r1[l], c.norm_eps)
            self._lin_fwd(self.h1[l], f"l{l}.wqkv", self.qkv)
            ops.rope_split(self.qkv, self.cos, self.sin, B, T, H, self.Qh[l], self.Kh[l],
                           self.Vh[l])
            self._attn_fwd(l, scale)
            ops.heads_merge(self.Oh[l], B, T, H, self.o[l])
            self._lin_fwd(self.o[l], f"l{l}.wo", x_mid, res=x_in)
            ops.norm_fwd(x_mid, pw(f"l{l}.mlp_norm"), self.h2[l], self.r2[l], c.norm_eps)
            self._lin_fwd(self.h2[l], f"l{l}.wgu", self.gu[l])
            ops.swiglu_fwd(self.gu[l], self.a[l])
            self._lin_fwd(self.a[l], f"l{l}.wdown", x_out, res=x_mid)
        ops.norm_fwd(self.xs[2 * L], pw("final_norm"), self.hf, self.rf, c.norm_eps)
        self._lin_fwd(self.hf, "head", self.logits)
        ops.ce(self.logits, tgt, self.losses)
        # ---------------- backward (adjoints + their tangents)
        self._linear_bwd("head", self.hf, self.logits, self.gh)
        ops.norm_bwd(self.xs[2 * L], self.gh, pw("final_norm"), self.rf, self.gx,
                     pg("final_norm"), accumulate=False)
        for l in reversed(range(L)):
            x_in, x_mid = self.xs[2 * l], self.xs[2 * l + 1]
            # MLP branch: gx is the adjoint of x_out (= of the wdown output and of x_mid)
            self._linear_bwd(f"l{l}.wdown", self.a[l], self.gx, self.ga)
            ops.swiglu_bwd(self.gu[l], self.ga, self.ggu)
            self._linear_bwd(f"l{l}.wgu", self.h2[l], self.ggu, self.gh)
            ops.norm_bwd(x_mid, self.gh, pw(f"l{l}.mlp_norm"), self.r2[l], self.gx,
                         pg(f"l{l}.mlp_norm"), accumulate=True)
            # attention branch
            self._linear_bwd(f"l{l}.wo", self.o[l], self.gx, self.go)
            ops.heads_split(self.go, B, T, H, self.GOh)
            self._attn_bwd(l, scale)
            ops.rope_merge(self.GQh, self.GKh, self.GVh, self.cos, self.sin, B, T, H,
                           self.gqkv)
            self._linear_bwd(f"l{l}.wqkv", self.h1[l], self.gqkv, self.gh)
            ops.norm_bwd(x_in, self.gh, pw(f"l{l}.attn_norm"), self.r1[l], self.gx,
                         pg(f"l{l}.attn_norm"), accumulate=True)
        ops.embed_bwd(tok, self.gx, pg("embed"))
        if Gl is not None:
            for dst, src in zip(Gl, Gs):
                dst.copy_(src)
        return self.losses
