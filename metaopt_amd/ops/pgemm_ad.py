"""Population GEMM with forward- AND reverse-mode derivatives, for second-order use.

``matmul(a, b, ta=False, tb=False)`` = ``op(a) @ op(b)`` per trial (``ta``: ``a`` is stored
``[K, M]``; ``tb``: ``b`` is stored ``[N, K]``) as a ``torch.autograd.Function`` that
``torch.func`` can transform: its ``jvp`` and its ``backward`` are themselves written with
``matmul``, so ``torch.func.jvp(torch.func.grad(f))`` -- the Hessian-vector products of the
unrolled hypergradient (K11, ``models/hyper.py``) -- runs every GEMM of the forward, the
backward AND the tangent propagation on the hand-written MFMA kernel (``csrc/pgemm.hip``),
operands read in their stored layout (no transposed copies).

On the GPU the operands are rounded to bf16 and accumulated in f32 (the kernel's contract; f32
operands are rounded as the kernel stages them and the f32 result is returned unrounded); on
CPU the same Function computes in fp32 with ``torch.bmm`` (the exact reference of the tests).

Derivatives of ``C = A B`` (``A = op(a)``, ``B = op(b)``):
* tangent: ``dC = dA B + A dB``;
* adjoint: ``gA = g B^T``, ``gB = A^T g`` -- mapped back to the stored layouts of ``a``/``b``.
"""
from __future__ import annotations

import torch


def _mm(a: torch.Tensor, b: torch.Tensor, ta: bool, tb: bool) -> torch.Tensor:
    if a.device.type == "cuda":
        from .gemm import pgemm
        if a.dtype == torch.float32 and b.dtype == torch.float32:
            # f32 operands are rounded to bf16 inside the kernel and the f32 accumulators come
            # back as they are: no cast kernels around the GEMM
            return pgemm(a.contiguous(), b.contiguous(), ta=ta, tb=tb)
        a16 = a.to(torch.bfloat16).contiguous()
        b16 = b.to(torch.bfloat16).contiguous()
        return pgemm(a16, b16, ta=ta, tb=tb).to(a.dtype)
    aa = a.transpose(1, 2) if ta else a
    bb = b.transpose(1, 2) if tb else b
    return torch.bmm(aa, bb)


class _MatmulPG(torch.autograd.Function):
    @staticmethod
    def forward(a, b, ta, tb):
        return _mm(a, b, ta, tb)

    @staticmethod
    def setup_context(ctx, inputs, output):
        a, b, ta, tb = inputs
        ctx.save_for_backward(a, b)
        ctx.save_for_forward(a, b)
        ctx.ta, ctx.tb = ta, tb

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ta, tb = ctx.ta, ctx.tb
        ga = gb = None
        if ctx.needs_input_grad[0]:
            # gA = g B^T; a stored as A^T when ta: ga = (g B^T)^T = B g^T
            ga = matmul(b, g, tb, True) if ta else matmul(g, b, False, not tb)
        if ctx.needs_input_grad[1]:
            # gB = A^T g; b stored as B^T when tb: gb = (A^T g)^T = g^T A
            gb = matmul(g, a, True, ta) if tb else matmul(a, g, not ta, False)
        return ga, gb, None, None

    @staticmethod
    def vmap(info, in_dims, a, b, ta, tb):
        """Batching rule: the vmapped dimension folds into the population dimension, so a
        batch of tangents (K11: one per hyper-parameter) is ONE population GEMM."""
        B = info.batch_size

        def fold(x, d):
            x = x.unsqueeze(0).expand(B, *x.shape) if d is None else x.movedim(d, 0)
            return x.reshape(B * x.shape[1], *x.shape[2:])

        out = matmul(fold(a, in_dims[0]), fold(b, in_dims[1]), ta, tb)
        return out.view(B, -1, *out.shape[1:]), 0

    @staticmethod
    def jvp(ctx, da, db, _ta, _tb):
        a, b = ctx.saved_tensors
        out = None
        if da is not None:
            out = matmul(da, b, ctx.ta, ctx.tb)
        if db is not None:
            t = matmul(a, db, ctx.ta, ctx.tb)
            out = t if out is None else out + t
        return out


def matmul(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False):
    """Differentiable (to any order, forward or reverse) ``op(a) @ op(b)`` for [P, ., .]."""
    return _MatmulPG.apply(a, b, ta, tb)
