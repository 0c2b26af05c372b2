"""Population-LM operators: HIP kernels (gfx950) behind autograd Functions, plus fp32 PyTorch
references of the same math (the CPU backend and the numerics oracle of tests/test_lm_gpu.py).

Every op carries a leading population dimension.  Row layout: activations are ``[R, d]`` with
``R = P * B * T`` rows ordered (trial, sequence, position); per-trial parameters are ``[P, ...]``.
Attention uses head-major ``[P * B, H, T, 64]`` for Q/K/V and the row layout for its output.

On a GPU the HIP path is the only path: a missing kernel library raises
(:class:`~metaopt_amd.ops._lib.KernelLibraryError`) instead of falling back to PyTorch.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Tuple

import numpy as np
import torch

from . import _lib

c_void_p, c_int, c_float, c_int64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64

_lib.register_signatures({
    "mopt_attn_fwd": ([c_void_p] * 5 + [c_int, c_int, c_int, c_float, c_void_p], c_int),
    "mopt_attn_bwd": ([c_void_p] * 10 + [c_int, c_int, c_int, c_float] + [c_void_p] * 4, c_int),
    "mopt_rmsnorm_fwd": ([c_void_p] * 4 + [c_int, c_int, c_int, c_float, c_void_p], c_int),
    "mopt_rmsnorm_bwd": ([c_void_p] * 6 + [c_int, c_int, c_int, c_void_p], c_int),
    "mopt_add_rmsnorm_fwd": ([c_void_p] * 6 + [c_int, c_int, c_int, c_float, c_void_p], c_int),
    "mopt_rmsnorm_bwd_res": ([c_void_p] * 7 + [c_int, c_int, c_int, c_void_p], c_int),
    "mopt_rmsnorm_dw_splits": ([c_int], c_int),
    "mopt_rmsnorm_dw16": ([c_void_p] * 5 + [c_int, c_int, c_int, c_void_p], c_int),
    "mopt_rmsnorm_bwd_dw16": ([c_void_p] * 8 + [c_int, c_int, c_int, c_void_p], c_int),
    "mopt_rope_fwd": ([c_void_p] * 6 + [c_int] * 4 + [c_void_p], c_int),
    "mopt_rope_bwd": ([c_void_p] * 6 + [c_int] * 4 + [c_void_p], c_int),
    "mopt_pgemm_qkv_rope": ([c_void_p] * 5 + [c_int] * 7 + [c_int64, c_int64, c_int, c_void_p],
                            c_int),
    "mopt_swiglu_fwd": ([c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p], c_int),
    "mopt_swiglu_bwd": ([c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p], c_int),
    "mopt_pgemm_swiglu": ([c_void_p] * 4 + [c_int] * 8 + [c_int64] * 4 + [c_int, c_void_p],
                          c_int),
    "mopt_ce_fwd_bwd": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int,
                         c_void_p], c_int),
    "mopt_embed_fwd": ([c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p],
                       c_int),
    "mopt_embed_bwd": ([c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p],
                       c_int),
    "mopt_cast_bf16": ([c_void_p, c_void_p, c_int64, c_void_p], c_int),
    "mopt_embed_bwd_sorted": ([c_void_p] * 4 + [c_int64, c_int, c_int64, c_void_p], c_int),
    "mopt_embed_sort": ([c_void_p] * 3 + [c_int] * 3 + [c_void_p], c_int),
    "mopt_embed_zero_rows": ([c_void_p] * 2 + [c_int64, c_int, c_int64, c_void_p], c_int),
    "mopt_adamw_multi": ([c_void_p, c_void_p, c_int] + [c_void_p] * 7 + [c_int] * 4 + [c_void_p],
                         c_int),
    "mopt_sgd_multi": ([c_void_p, c_void_p, c_int] + [c_void_p] * 6 + [c_int] * 3 + [c_void_p],
                       c_int),
})

LM_HP_DTYPE = np.dtype([("lr", "<f4"), ("b1", "<f4"), ("b2", "<f4"), ("eps", "<f4"),
                        ("wd", "<f4"), ("max_norm", "<f4"), ("t", "<i4"), ("pad", "<i4")])
SEG_DTYPE = np.dtype([("off", "<i8"), ("numel", "<i8")])
SEGCHUNK_DTYPE = np.dtype([("seg", "<i4"), ("trial", "<i4"), ("start", "<i8")])
ADAM_CHUNK = 2048


_FORCE_REF = {x.strip() for x in os.environ.get("MOPT_LM_REFERENCE", "").split(",") if x.strip()}


def _hip(t: torch.Tensor, op: str = "") -> bool:
    """HIP kernel on a GPU.  ``MOPT_LM_REFERENCE=all`` or ``=attn,ce,...`` explicitly selects the
    PyTorch reference for those ops (a debugging / bisection aid; never a silent fallback)."""
    if t.device.type != "cuda":
        return False
    return not (_FORCE_REF and ("all" in _FORCE_REF or op in _FORCE_REF))


def _call(name, *args):
    lib = _lib.get_lib()
    _lib.check(getattr(lib, name)(*args), name)


def _stream(t):
    return _lib.stream_ptr(t.device)


def _p(t):
    return t.data_ptr()


# ============================================================================ references (fp32)
def rmsnorm_ref(x, w, rows_per_trial, eps=1e-5):
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    wf = w.float().repeat_interleave(rows_per_trial, 0)
    return (xf * r * wf).to(x.dtype)


def rope_tables(T: int, base: float = 10000.0, device=None):
    inv = base ** (-torch.arange(0, 32, dtype=torch.float64) / 32.0)
    ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
    return (torch.cos(ang).float().contiguous().to(device),
            torch.sin(ang).float().contiguous().to(device))


def rope_split_ref(qkv, cos, sin, T, H, il=False):
    """q, k, v heads [B', H, T, 64] of the QKV activation [B' T, 3 H 64], q and k rotated by
    rotate-half pairs (j, j + 32) or (``il``) interleaved pairs (2j, 2j + 1) at angle j."""
    R = qkv.shape[0]
    Bp = R // T
    x = qkv.float().view(Bp, T, 3, H, 64).permute(2, 0, 3, 1, 4)  # [3, B', H, T, 64]
    q, k, v = x[0], x[1], x[2]

    def rot(t):
        c, s = cos[None, None], sin[None, None]
        if il:
            t1, t2 = t[..., 0::2], t[..., 1::2]
            return torch.stack([t1 * c - t2 * s, t2 * c + t1 * s], -1).flatten(-2)
        t1, t2 = t[..., :32], t[..., 32:]
        return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], -1)
    return (rot(q).to(qkv.dtype).contiguous(), rot(k).to(qkv.dtype).contiguous(),
            v.to(qkv.dtype).contiguous())


def attention_ref(q, k, v, scale):
    """Causal softmax attention in fp32; returns [B', T, H, 64] flattened to rows."""
    Bp, H, T, Dh = q.shape
    s = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) * scale
    mask = torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    o = torch.einsum("bhqk,bhkd->bhqd", s.softmax(-1), v.float())
    return o.permute(0, 2, 1, 3).reshape(Bp * T, H * Dh).to(q.dtype)


def swiglu_split(gu, il=False):
    """(gate, up) of a gate/up activation: two halves, or (``il``) interleaved 16-column groups
    [g0..g15 u0..u15 g16..] -- the layout of the fused gate/up GEMM epilogue (pgemm.hip EPI)."""
    F = gu.shape[-1] // 2
    if not il:
        return gu[..., :F], gu[..., F:]
    v = gu.reshape(*gu.shape[:-1], F // 16, 2, 16)
    return v[..., 0, :].reshape(*gu.shape[:-1], F), v[..., 1, :].reshape(*gu.shape[:-1], F)


def swiglu_ref(gu, il=False):
    g, u = swiglu_split(gu.float(), il)
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


def ce_ref(logits, labels, rows_per_trial):
    """Per-trial SUM of token losses, fp32."""
    lz = torch.nn.functional.cross_entropy(logits.float(), labels.long(), reduction="none")
    return lz.view(-1, rows_per_trial).sum(1)


def embed_ref(tok, table, rows_per_trial):
    P, V, d = table.shape
    p = torch.arange(tok.numel(), device=tok.device) // rows_per_trial
    return table[p, tok.long()]


# ============================================================================ autograd Functions
def _grad_view(t):
    """The leaf's preset ``.grad`` (a view of the flat bf16 gradient buffer) when the kernels can
    write the gradient there directly -- autograd then has nothing to accumulate."""
    if t.requires_grad and t.is_leaf and t.grad is not None and t.grad.is_contiguous() and \
            t.grad.dtype == torch.bfloat16:
        return t.grad
    return None


def _dw_out(dw32, gw, dtype, stream_of):
    """f32 weight gradient -> the flat buffer (returns None) or a tensor for autograd."""
    if gw is not None:
        _call("mopt_cast_bf16", _p(dw32), _p(gw), dw32.numel(), _stream(stream_of))
        return None
    return dw32.to(dtype)


# RMSNorm backward with the weight gradient's partial sums in the dx pass (csrc/lm_ops.hip
# rmsnorm_bwd_dxdw_kernel); MOPT_NORM_DXDW=0: the separate partial pass, for A/B runs
_NORM_DXDW = os.environ.get("MOPT_NORM_DXDW", "1") != "0"


def _norm_bwd_dw(x, w, dy, dres, rstd, dx, gw, rows_per_trial):
    """dx (+ dres) and the weight gradient into the flat bf16 view ``gw`` in one pass over x and
    dy (+ the partials' reduce)."""
    R, d = x.shape
    S = _lib.get_lib().mopt_rmsnorm_dw_splits(rows_per_trial)
    part = torch.empty(S * (R // rows_per_trial) * d, dtype=torch.float32, device=x.device)
    _call("mopt_rmsnorm_bwd_dw16", _p(x), _p(w), _p(dy), _p(dres) if dres is not None else None,
          _p(rstd), _p(dx), _p(part), _p(gw), R, d, rows_per_trial, _stream(x))


def _norm_dw(x, dy, rstd, gw, rows_per_trial):
    """RMSNorm weight gradient written into the flat bf16 gradient view ``gw``: per-slice f32
    partials, then one reduce that writes bf16 (no zero fill, no atomics, no cast kernel).
    ``x`` is the norm's input.  Returns None (autograd has nothing to accumulate)."""
    R, d = x.shape
    S = _lib.get_lib().mopt_rmsnorm_dw_splits(rows_per_trial)
    part = torch.empty(S * (R // rows_per_trial) * d, dtype=torch.float32, device=x.device)
    _call("mopt_rmsnorm_dw16", _p(x), _p(dy), _p(rstd), _p(part), _p(gw), R, d,
          rows_per_trial, _stream(x))
    return None


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, rows_per_trial, eps):
        R, d = x.shape
        y = torch.empty_like(x)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        _call("mopt_rmsnorm_fwd", _p(x), _p(w), _p(y), _p(rstd), R, d, rows_per_trial, eps,
              _stream(x))
        ctx.save_for_backward(x, w, rstd)
        ctx.rpt = rows_per_trial
        ctx.gw = _grad_view(w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        R, d = x.shape
        dx = torch.empty_like(x)
        if ctx.gw is not None and _NORM_DXDW:
            _norm_bwd_dw(x, w, dy, None, rstd, dx, ctx.gw, ctx.rpt)
            return dx, None, None, None
        if ctx.gw is not None:
            _call("mopt_rmsnorm_bwd", _p(x), _p(w), _p(dy), _p(rstd), _p(dx), None, R, d,
                  ctx.rpt, _stream(x))
            return dx, _norm_dw(x, dy, rstd, ctx.gw, ctx.rpt), None, None
        dw32 = torch.zeros(w.shape, dtype=torch.float32, device=x.device)
        _call("mopt_rmsnorm_bwd", _p(x), _p(w), _p(dy), _p(rstd), _p(dx), _p(dw32), R, d,
              ctx.rpt, _stream(x))
        return dx, _dw_out(dw32, ctx.gw, w.dtype, x), None, None


def rmsnorm(x, w, rows_per_trial, eps=1e-5):
    if _hip(x, "rmsnorm"):
        return _RMSNorm.apply(x.contiguous(), w.contiguous(), rows_per_trial, eps)
    return rmsnorm_ref(x, w, rows_per_trial, eps)


class _AddRMSNorm(torch.autograd.Function):
    """(x + delta, rmsnorm(x + delta)) in one pass; the backward returns one gradient for both
    summands: the norm's dx plus the gradient that reached the sum directly, also one pass."""

    @staticmethod
    def forward(ctx, x, delta, w, rows_per_trial, eps):
        R, d = x.shape
        y = torch.empty_like(x)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        if delta is None:              # rmsnorm_pass: x itself is the sum
            xs = x
            _call("mopt_rmsnorm_fwd", _p(x), _p(w), _p(y), _p(rstd), R, d, rows_per_trial, eps,
                  _stream(x))
        else:
            xs = torch.empty_like(x)
            _call("mopt_add_rmsnorm_fwd", _p(x), _p(delta), _p(xs), _p(w), _p(y), _p(rstd), R, d,
                  rows_per_trial, eps, _stream(x))
        ctx.has_delta = delta is not None
        # an unused sum (the last norm's) reaches the backward as None, not a zero-filled [R, d]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(xs, w, rstd)
        ctx.rpt = rows_per_trial
        ctx.gw = _grad_view(w)
        return xs, y

    @staticmethod
    def backward(ctx, dxs, dy):
        xs, w, rstd = ctx.saved_tensors
        R, d = xs.shape
        if dy is None:
            dd = dxs if ctx.has_delta else None
            if ctx.gw is not None:
                ctx.gw.zero_()
                return dxs, dd, None, None, None
            return dxs, dd, torch.zeros_like(w), None, None
        dy = dy.contiguous()
        dres = dxs.contiguous() if dxs is not None else None
        dx = torch.empty_like(xs)
        dd = dx if ctx.has_delta else None
        if ctx.gw is not None and _NORM_DXDW:
            _norm_bwd_dw(xs, w, dy, dres, rstd, dx, ctx.gw, ctx.rpt)
            return dx, dd, None, None, None
        dw32 = None if ctx.gw is not None else \
            torch.zeros(w.shape, dtype=torch.float32, device=xs.device)
        _call("mopt_rmsnorm_bwd_res", _p(xs), _p(w), _p(dy),
              _p(dres) if dres is not None else None, _p(rstd), _p(dx),
              _p(dw32) if dw32 is not None else None, R, d, ctx.rpt, _stream(xs))
        if ctx.gw is not None:
            return dx, dd, _norm_dw(xs, dy, rstd, ctx.gw, ctx.rpt), None, None
        return dx, dd, dw32.to(w.dtype), None, None


def add_rmsnorm(x, delta, w, rows_per_trial, eps=1e-5):
    """Residual add fused into the following pre-norm: returns ``(x + delta, rmsnorm(x + delta))``."""
    if _hip(x, "add_rmsnorm"):
        return _AddRMSNorm.apply(x.contiguous(), delta.contiguous(), w.contiguous(),
                                 rows_per_trial, eps)
    xs = x + delta
    return xs, rmsnorm_ref(xs, w, rows_per_trial, eps)


def rmsnorm_pass(x, w, rows_per_trial, eps=1e-5):
    """``(x, rmsnorm(x))``: the norm's input passed through, so a gradient that reaches ``x``
    through its other uses joins the norm's backward pass (the ``dres`` addend of
    :class:`_AddRMSNorm`) instead of an autograd accumulation kernel."""
    if _hip(x, "rmsnorm"):
        return _AddRMSNorm.apply(x.contiguous(), None, w.contiguous(), rows_per_trial, eps)
    return x, rmsnorm_ref(x, w, rows_per_trial, eps)


class _RopeSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, T, H):
        R = qkv.shape[0]
        Bp = R // T
        shape = (Bp, H, T, 64)
        q = torch.empty(shape, dtype=qkv.dtype, device=qkv.device)
        k, v = torch.empty_like(q), torch.empty_like(q)
        _call("mopt_rope_fwd", _p(qkv), _p(cos), _p(sin), _p(q), _p(k), _p(v), R, T, H, 0,
              _stream(qkv))
        ctx.save_for_backward(cos, sin)
        ctx.dims = (R, T, H, qkv.shape)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        R, T, H, shape = ctx.dims
        dqkv = torch.empty(shape, dtype=dq.dtype, device=dq.device)
        _call("mopt_rope_bwd", _p(dq.contiguous()), _p(dk.contiguous()), _p(dv.contiguous()),
              _p(cos), _p(sin), _p(dqkv), R, T, H, 0, _stream(dq))
        return dqkv, None, None, None, None


def rope_split(qkv, cos, sin, T, H):
    if _hip(qkv, "rope"):
        return _RopeSplit.apply(qkv.contiguous(), cos, sin, T, H)
    return rope_split_ref(qkv, cos, sin, T, H)


class _QKVRope(torch.autograd.Function):
    """q, k, v = rope(h @ wqkv) per trial with interleaved RoPE pairs: the big-tile GEMM writes
    the rotated heads in its epilogue (csrc/pgemm.hip EPI 3; no QKV activation, no RoPE pass).
    Backward: the inverse rotation back into the [rows, 3 d] gradient, then its two GEMMs."""

    @staticmethod
    def forward(ctx, h, w, cos, sin, T, H, g_w):
        buf = _qkv_heads(h, w, cos, sin, T, H)
        ctx.save_for_backward(h, w, cos, sin)
        ctx.dims = (T, H)
        ctx.g_w = g_w
        return buf[0], buf[1], buf[2]

    @staticmethod
    def backward(ctx, dq, dk, dv):
        from .gemm import pgemm
        h, w, cos, sin = ctx.saved_tensors
        T, H = ctx.dims
        P, R, d = h.shape
        dqkv = torch.empty(P, R, 3 * d, dtype=h.dtype, device=h.device)
        _call("mopt_rope_bwd", _p(dq.contiguous()), _p(dk.contiguous()), _p(dv.contiguous()),
              _p(cos), _p(sin), _p(dqkv), P * R, T, H, 1, _stream(h))
        dw = None
        if ctx.g_w is not None:
            pgemm(h, dqkv, ta=True, out=ctx.g_w)
        else:
            dw = pgemm(h, dqkv, ta=True)
        return pgemm(dqkv, w, tb=True), dw, None, None, None, None, None


def _qkv_heads(h, w, cos, sin, T, H):
    """[3, B', H, T, 64] q, k, v heads of h @ w with interleaved RoPE (the EPI 3 GEMM, or the
    GEMM + the RoPE kernel on shapes without a big tile)."""
    from .gemm import LARGE_TILES, pgemm, plan
    P, R, d = h.shape
    buf = torch.empty(3, P * (R // T), H, T, 64, dtype=h.dtype, device=h.device)
    cfg, splits, _ = plan(P, R, 3 * d, d)
    rc = 801
    if cfg in LARGE_TILES and splits == 1 and R % T == 0:
        rc = _lib.get_lib().mopt_pgemm_qkv_rope(
            _p(h), _p(w), _p(buf), _p(cos), _p(sin), P, R, d, T, H, h.stride(1), w.stride(1),
            h.stride(0), w.stride(0), cfg, _stream(h))
    if rc == 801:
        qkv = pgemm(h, w)
        _call("mopt_rope_fwd", _p(qkv), _p(cos), _p(sin), _p(buf[0]), _p(buf[1]), _p(buf[2]),
              P * R, T, H, 1, _stream(h))
    else:
        _lib.check(rc, "mopt_pgemm_qkv_rope")
    return buf


class _QKVRopeAttention(torch.autograd.Function):
    """Causal attention over rope(h @ wqkv) in one autograd node: the QKV GEMM writes the rotated
    heads (EPI 3), and the attention backward writes the QKV activation's gradient with the
    inverse RoPE applied (no dQ / dK / dV buffers, no RoPE-backward pass), then the projection's
    two GEMMs."""

    @staticmethod
    def forward(ctx, h, w, cos, sin, T, H, scale, g_w):
        P, R, d = h.shape
        buf = _qkv_heads(h, w, cos, sin, T, H)
        q, k, v = buf[0], buf[1], buf[2]
        Bp = P * (R // T)
        o = torch.empty(Bp * T, H * 64, dtype=h.dtype, device=h.device)
        lse = torch.empty(Bp * H, T, dtype=torch.float32, device=h.device)
        _call("mopt_attn_fwd", _p(q), _p(k), _p(v), _p(o), _p(lse), Bp * H, T, H, scale,
              _stream(h))
        ctx.save_for_backward(h, w, cos, sin, buf, o, lse)
        ctx.meta = (T, H, scale)
        ctx.g_w = g_w
        return o

    @staticmethod
    def backward(ctx, do):
        from .gemm import pgemm
        h, w, cos, sin, buf, o, lse = ctx.saved_tensors
        T, H, scale = ctx.meta
        P, R, d = h.shape
        do = do.contiguous()
        dqkv = torch.empty(P, R, 3 * d, dtype=h.dtype, device=h.device)
        dsum = torch.empty_like(lse)
        _call("mopt_attn_bwd", _p(buf[0]), _p(buf[1]), _p(buf[2]), _p(o), _p(do), _p(lse),
              _p(dsum), None, None, None, P * (R // T) * H, T, H, scale, _p(dqkv), _p(cos),
              _p(sin), _stream(h))
        dw = None
        if ctx.g_w is not None:
            pgemm(h, dqkv, ta=True, out=ctx.g_w)
        else:
            dw = pgemm(h, dqkv, ta=True)
        return pgemm(dqkv, w, tb=True), dw, None, None, None, None, None, None


def qkv_rope_attention(h, w, cos, sin, T, H, scale=None):
    """Causal self-attention output [B' T, H 64] of the heads rope(h @ w) (interleaved RoPE):
    h [P, R, d], w [P, d, 3 d]."""
    scale = 0.125 if scale is None else scale            # head dim 64
    if _hip(h, "attn") and _hip(h, "rope"):
        return _QKVRopeAttention.apply(h.contiguous(), w.contiguous(), cos, sin, T, H, scale,
                                       _grad_view(w))
    q, k, v = qkv_rope(h, w, cos, sin, T, H)
    return attention_ref(q, k, v, scale) if not _hip(h, "attn") else attention(q, k, v, scale)


def qkv_rope(h, w, cos, sin, T, H):
    """(q, k, v) heads [B', H, T, 64] of ``h [P, R, d] @ w [P, d, 3 d]`` with interleaved-pair
    RoPE on q and k (the LM's attention input)."""
    if _hip(h, "rope"):
        return _QKVRope.apply(h.contiguous(), w.contiguous(), cos, sin, T, H, _grad_view(w))
    P, R, d = h.shape
    return rope_split_ref(torch.bmm(h, w).reshape(P * R, 3 * d), cos, sin, T, H, il=True)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale):
        Bp, H, T, Dh = q.shape
        if Dh != 64 or T % 64:
            raise ValueError("attention kernel: head dim 64, T multiple of 64")
        o = torch.empty(Bp * T, H * Dh, dtype=q.dtype, device=q.device)
        lse = torch.empty(Bp * H, T, dtype=torch.float32, device=q.device)
        _call("mopt_attn_fwd", _p(q), _p(k), _p(v), _p(o), _p(lse), Bp * H, T, H, scale,
              _stream(q))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        Bp, H, T, _ = q.shape
        do = do.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dsum = torch.empty_like(lse)
        _call("mopt_attn_bwd", _p(q), _p(k), _p(v), _p(o), _p(do), _p(lse), _p(dsum), _p(dq),
              _p(dk), _p(dv), Bp * H, T, H, ctx.scale, None, None, None, _stream(q))
        return dq, dk, dv, None


def attention(q, k, v, scale=None):
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if _hip(q, "attn"):
        return _Attention.apply(q, k, v, scale)
    return attention_ref(q, k, v, scale)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        rows, F2 = gu.shape[0] * (gu.shape[1] if gu.dim() == 3 else 1), gu.shape[-1]
        h = torch.empty(*gu.shape[:-1], F2 // 2, dtype=gu.dtype, device=gu.device)
        _call("mopt_swiglu_fwd", _p(gu), _p(h), rows, F2 // 2, 0, _stream(gu))
        ctx.save_for_backward(gu)
        return h

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        rows, F2 = gu.numel() // gu.shape[-1], gu.shape[-1]
        dgu = torch.empty_like(gu)
        _call("mopt_swiglu_bwd", _p(gu), _p(dh.contiguous()), _p(dgu), rows, F2 // 2, 0,
              _stream(gu))
        return dgu


def swiglu(gu):
    if _hip(gu, "swiglu"):
        return _SwiGLU.apply(gu.contiguous())
    return swiglu_ref(gu)


def _swiglu_gemm(a, b, c, x):
    """``c = a @ b`` (the gate / up product) with the SwiGLU activation ``x`` written by the
    big-tile GEMM's epilogue (csrc/pgemm.hip EPI 1); False when the shape's plan has no big tile
    or splits K (the caller runs the GEMM and the swiglu kernel)."""
    from .gemm import LARGE_TILES, plan
    P, M, K = a.shape
    N = b.shape[2]
    cfg, splits, _ = plan(P, M, N, K)
    if cfg not in LARGE_TILES or splits != 1 or N % 32:
        return False
    rc = _lib.get_lib().mopt_pgemm_swiglu(
        _p(a), _p(b), _p(c), _p(x), P, M, N, K, a.stride(1), b.stride(1), c.stride(1),
        x.stride(1), a.stride(0), b.stride(0), c.stride(0), x.stride(0), cfg, _stream(a))
    if rc == 801:                          # hipErrorNotSupported
        return False
    _lib.check(rc, "mopt_pgemm_swiglu")
    return True


class _SwiGLUMLP(torch.autograd.Function):
    """``swiglu(h @ wgu) @ wdown`` of every trial, gate / up columns interleaved in 16-column
    groups.  Forward: the gate/up GEMM writes the activation in its epilogue (no SwiGLU pass).
    The weight gradients go straight into the flat gradient buffer's views when given."""

    @staticmethod
    def forward(ctx, h, wgu, wdown, g_gu, g_down):
        from .gemm import pgemm
        P, R, _ = h.shape
        F = wdown.shape[1]
        gu = torch.empty(P, R, 2 * F, dtype=h.dtype, device=h.device)
        a = torch.empty(P, R, F, dtype=h.dtype, device=h.device)
        if not _swiglu_gemm(h, wgu, gu, a):
            pgemm(h, wgu, out=gu)
            _call("mopt_swiglu_fwd", _p(gu), _p(a), P * R, F, 1, _stream(h))
        ctx.save_for_backward(h, wgu, wdown, gu, a)
        ctx.grads = (g_gu, g_down)
        return pgemm(a, wdown)

    @staticmethod
    def backward(ctx, dy):
        from .gemm import pgemm
        h, wgu, wdown, gu, a = ctx.saved_tensors
        g_gu, g_down = ctx.grads
        dy = dy.contiguous()
        P, R, _ = h.shape
        F = wdown.shape[1]
        dwdown = dwgu = None
        if g_down is not None:
            pgemm(a, dy, ta=True, out=g_down)
        else:
            dwdown = pgemm(a, dy, ta=True)
        # (a dgu epilogue on the dh GEMM -- g, u loaded per fragment -- doubled that GEMM and
        # saved nothing: profiles/round4.md; the backward keeps the separate pass)
        dgu = torch.empty_like(gu)
        dh = pgemm(dy, wdown, tb=True)
        _call("mopt_swiglu_bwd", _p(gu), _p(dh), _p(dgu), P * R, F, 1, _stream(dy))
        if g_gu is not None:
            pgemm(h, dgu, ta=True, out=g_gu)
        else:
            dwgu = pgemm(h, dgu, ta=True)
        dh_in = pgemm(dgu, wgu, tb=True)
        return dh_in, dwgu, dwdown, None, None


def swiglu_mlp(h, wgu, wdown):
    """``swiglu(h @ wgu) @ wdown`` per trial: h [P, R, d], wgu [P, d, 2F] (gate / up in
    interleaved 16-column groups, :func:`swiglu_split`), wdown [P, F, d]."""
    if _hip(h, "swiglu"):
        return _SwiGLUMLP.apply(h.contiguous(), wgu.contiguous(), wdown.contiguous(),
                                _grad_view(wgu), _grad_view(wdown))
    return torch.bmm(swiglu_ref(torch.bmm(h, wgu), il=True), wdown)


class _CrossEntropy(torch.autograd.Function):
    """Per-trial sum of token losses; the gradient (softmax - onehot) is written over the
    logits buffer in the forward pass (the logits are not needed afterwards)."""

    @staticmethod
    def forward(ctx, logits, labels, rows_per_trial, grad_scale, unit_weights):
        ctx.unit_weights = unit_weights
        R, V = logits.shape[-2] * (logits.shape[0] if logits.dim() == 3 else 1), logits.shape[-1]
        P = R // rows_per_trial
        loss = torch.zeros(P, dtype=torch.float32, device=logits.device)
        _call("mopt_ce_fwd_bwd", _p(logits), _p(labels), _p(loss), R, V, rows_per_trial,
              grad_scale, 1, _stream(logits))
        ctx.save_for_backward(logits)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (dlogits,) = ctx.saved_tensors
        if ctx.unit_weights:
            # the caller differentiates sum_p loss_p: d/dloss_p = 1, no pass over the logits
            # (and no host-side check, so the step can be captured in a HIP graph)
            return dlogits, None, None, None, None
        P = dloss.numel()
        g = dlogits.view(P, -1, dlogits.shape[-1]) * dloss.view(P, 1, 1).to(dlogits.dtype)
        return g.view_as(dlogits), None, None, None, None


def cross_entropy(logits, labels, rows_per_trial, grad_scale=1.0, unit_weights=False):
    """Returns the per-trial SUM of token losses [P] (fp32).  ``grad_scale`` multiplies the
    gradient written for the backward (``1 / rows_per_trial`` gives mean-loss gradients).
    ``unit_weights=True`` promises the result is only differentiated through ``loss.sum()``."""
    if _hip(logits, "ce"):
        return _CrossEntropy.apply(logits.contiguous(), labels.contiguous(), rows_per_trial,
                                   grad_scale, unit_weights)
    loss = ce_ref(logits.reshape(-1, logits.shape[-1]), labels, rows_per_trial)
    return loss if grad_scale == 1.0 else _ScaledGrad.apply(loss, grad_scale)


class _ScaledGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


def ce_eval(logits, labels, rows_per_trial):
    """Loss sums without writing gradients (validation)."""
    if _hip(logits, "ce"):
        R, V = logits.numel() // logits.shape[-1], logits.shape[-1]
        loss = torch.zeros(R // rows_per_trial, dtype=torch.float32, device=logits.device)
        _call("mopt_ce_fwd_bwd", _p(logits.contiguous()), _p(labels.contiguous()), _p(loss), R, V,
              rows_per_trial, 1.0, 0, _stream(logits))
        return loss
    return ce_ref(logits.reshape(-1, logits.shape[-1]), labels, rows_per_trial)


#: rows per trial the in-LDS key sort takes (csrc/lm_ops.hip kEmbedSortMax)
EMBED_SORT_MAX = 8192
_EMBED_KEYS: dict = {}


def _embed_key_buffers(gw: torch.Tensor, R: int):
    """(keys, order) int64 [R] kept per table-gradient buffer across steps (and HIP-graph
    replays): ``keys`` holds the previous step's sorted keys, whose table rows are the only
    non-zero ones.  Created with keys = -1 (nothing to clear) outside any graph capture -- the
    population's eager warm-up steps run first; a first call inside a capture would record the
    -1 fill into the graph, so it falls back to the full clear (None)."""
    key = (gw.device, gw.data_ptr(), gw.numel(), R)
    buf = _EMBED_KEYS.get(key)
    if buf is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        gw.zero_()                      # the invariant's base case: every row zero
        buf = (torch.full((R,), -1, dtype=torch.int64, device=gw.device),
               torch.empty(R, dtype=torch.int64, device=gw.device))
        _EMBED_KEYS[key] = buf
    return buf


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, table, rows_per_trial):
        P, V, d = table.shape
        R = tok.numel()
        out = torch.empty(R, d, dtype=table.dtype, device=table.device)
        _call("mopt_embed_fwd", _p(tok), _p(table), _p(out), R, d, V, rows_per_trial,
              _stream(table))
        ctx.save_for_backward(tok)
        ctx.dims = (P, V, d, rows_per_trial, table.dtype)
        ctx.gw = _grad_view(table)
        return out

    @staticmethod
    def backward(ctx, dout):
        (tok,) = ctx.saved_tensors
        P, V, d, rpt, dtype = ctx.dims
        dout = dout.contiguous()
        if ctx.gw is not None:
            # sort the (trial, token) keys once (stable: deterministic sums) and let one wave per
            # run of equal keys write its row -- no f32 table, no atomics, no cast pass
            R = tok.numel()
            n = 1 << max(0, (rpt - 1).bit_length())
            buf = _embed_key_buffers(ctx.gw, R) if n <= EMBED_SORT_MAX else None
            if buf is None:            # rows per trial past the in-LDS sort: library sort
                trial = torch.arange(R, device=tok.device, dtype=torch.int64) // rpt
                keys, order = torch.sort(trial * V + tok.long(), stable=True)
                ctx.gw.zero_()
            else:
                # the rows the previous step wrote (every other row is zero), then this step's
                # keys sorted in place of them (csrc/lm_ops.hip embed_sort_kernel)
                keys, order = buf
                _call("mopt_embed_zero_rows", _p(keys), _p(ctx.gw), R, d, P * V, _stream(dout))
                _call("mopt_embed_sort", _p(tok), _p(keys), _p(order), P, rpt, V, _stream(dout))
            _call("mopt_embed_bwd_sorted", _p(keys), _p(order), _p(dout), _p(ctx.gw), R, d,
                  P * V, _stream(dout))
            return None, None, None
        d32 = torch.zeros(P, V, d, dtype=torch.float32, device=dout.device)
        _call("mopt_embed_bwd", _p(tok), _p(dout.contiguous()), _p(d32), tok.numel(), d, V, rpt,
              _stream(dout))
        d16 = torch.empty(P, V, d, dtype=dtype, device=dout.device)
        _call("mopt_cast_bf16", _p(d32), _p(d16), d32.numel(), _stream(dout))
        return None, d16, None


def embedding(tok, table, rows_per_trial):
    if _hip(table, "embed"):
        return _Embedding.apply(tok.contiguous(), table, rows_per_trial)
    return embed_ref(tok, table, rows_per_trial)


# ============================================================================ fused AdamW
class FlatOptimizer:
    """Fused per-trial optimizer over flat parameter buffers: AdamW (north-star kernel K6) or
    SGD-momentum (K5), with optional per-trial global-norm gradient clipping.

    ``segments``: [(offset, numel_per_trial)] of every parameter tensor inside the flat buffers,
    each tensor laid out ``[P, numel]``.  State: f32 master weights ``p32``, ``m`` (and ``v`` for
    AdamW); the bf16 working copy ``p16`` is rewritten by the same kernel; ``g16`` is the flat bf16
    gradient.  Hyper-parameters are per trial (``hp`` structured array, :data:`LM_HP_DTYPE`;
    SGD reads ``lr``, ``b1`` = momentum, ``wd``, ``max_norm``).  Work is listed as chunks of at
    most 2048 elements of ONE trial, so every lane knows its trial without a division.
    """

    def __init__(self, segments: List[Tuple[int, int]], P: int, device, kind: str = "adamw"):
        if kind not in ("adamw", "sgd"):
            raise ValueError(f"unknown optimizer {kind}")
        self.kind = kind
        self.P = P
        self.device = torch.device(device)
        segs = np.array(segments, dtype=SEG_DTYPE)
        chunks = []
        for j, (off, numel) in enumerate(segments):
            for p in range(P):
                starts = np.arange(p * numel, (p + 1) * numel, ADAM_CHUNK, dtype=np.int64)
                c = np.zeros(len(starts), dtype=SEGCHUNK_DTYPE)
                c["seg"], c["trial"], c["start"] = j, p, starts
                chunks.append(c)
        chunks = np.concatenate(chunks) if chunks else np.zeros(0, SEGCHUNK_DTYPE)
        self.segments = segments
        self.n_chunks = len(chunks)
        if self.device.type == "cuda":
            self._segs = _lib.upload_bytes(segs, self.device)
            self._chunks = _lib.upload_bytes(chunks, self.device)
            self._sumsq = torch.zeros(P, dtype=torch.float32, device=self.device)

    def step(self, master, p16, g16, m, v, hp: np.ndarray, hp_dev=None):
        """``master``: the f32 master weights, or (int16) the low halves of a split master whose
        high halves are the bf16 working copy ``p16`` (csrc/common.h split4).  ``hp_dev``: the
        hyper-parameters already on the device (graph replay); else ``hp`` is uploaded."""
        clip = int(bool((hp["max_norm"] > 0).any()))
        split = master.dtype == torch.int16
        if self.device.type == "cuda":
            if hp_dev is None:
                hp_dev = _lib.upload_bytes(hp, self.device)
            if self.kind == "adamw":
                _call("mopt_adamw_multi", _p(self._segs), _p(self._chunks), self.n_chunks,
                      _p(hp_dev), _p(self._sumsq), _p(master), _p(p16), _p(g16), _p(m), _p(v),
                      self.P, clip, int(m.dtype == torch.bfloat16), int(split),
                      _lib.stream_ptr(self.device))
            else:
                _call("mopt_sgd_multi", _p(self._segs), _p(self._chunks), self.n_chunks,
                      _p(hp_dev), _p(self._sumsq), _p(master), _p(p16), _p(g16), _p(m), self.P,
                      clip, int(split), _lib.stream_ptr(self.device))
            return
        from .reference import join_f32, split_f32
        p32 = join_f32(p16, master) if split else master
        if self.kind == "adamw":
            adamw_flat_ref(self.segments, self.P, p32, p16, g16, m, v, hp)
        else:
            sgd_flat_ref(self.segments, self.P, p32, p16, g16, m, hp)
        if split:
            hi, lo = split_f32(p32)
            p16.copy_(hi)
            master.copy_(lo)


FlatAdamW = FlatOptimizer


def _clip_scales(segments, P, g, hp):
    sumsq = torch.zeros(P, dtype=torch.float64)
    for off, numel in segments:
        sumsq += g[off:off + P * numel].view(P, numel).double().pow(2).sum(1).cpu()
    scales = []
    for p in range(P):
        s = 1.0
        if hp[p]["max_norm"] > 0:
            nrm = math.sqrt(float(sumsq[p]))
            if nrm > hp[p]["max_norm"]:
                s = float(hp[p]["max_norm"]) / (nrm + 1e-6)
        scales.append(s)
    return scales


def sgd_flat_ref(segments, P, p32, p16, g16, m, hp):
    """fp32 reference of the flat SGD-momentum update."""
    g = g16.float()
    scales = _clip_scales(segments, P, g, hp)
    for off, numel in segments:
        for p in range(P):
            h = hp[p]
            lo, hi = off + p * numel, off + (p + 1) * numel
            d = g[lo:hi] * scales[p] + float(h["wd"]) * p32[lo:hi]
            m[lo:hi].mul_(float(h["b1"])).add_(d)
            p32[lo:hi].sub_(float(h["lr"]) * m[lo:hi])
        sl = slice(off, off + P * numel)
        p16[sl] = p32[sl].to(p16.dtype)


def adamw_flat_ref(segments, P, p32, p16, g16, m, v, hp):
    """fp32 reference of the flat AdamW update (same clipping and bias correction)."""
    g = g16.float()
    scales = _clip_scales(segments, P, g, hp)
    for off, numel in segments:
        sl = slice(off, off + P * numel)
        for p in range(P):
            h = hp[p]
            lo, hi = off + p * numel, off + (p + 1) * numel
            gr = g[lo:hi] * scales[p]
            t = float(h["t"])
            bc1, bc2 = 1 - float(h["b1"]) ** t, 1 - float(h["b2"]) ** t
            w = p32[lo:hi]
            w.mul_(1 - float(h["lr"]) * float(h["wd"]))
            mf = m[lo:hi].float() * float(h["b1"]) + (1 - float(h["b1"])) * gr
            m[lo:hi] = mf.to(m.dtype)          # a bf16 first moment rounds once per update
            v[lo:hi].mul_(float(h["b2"])).addcmul_(gr, gr, value=1 - float(h["b2"]))
            denom = v[lo:hi].sqrt() / math.sqrt(bc2) + float(h["eps"])
            w.addcdiv_(mf, denom, value=-float(h["lr"]) / bc1)
        p16[sl] = p32[sl].to(p16.dtype)
