"""Population-batched GEMM with a backward that only issues NN-layout GEMMs.

``pbmm(a, b)`` = ``torch.bmm(a, b)`` (hipBLASLt strided-batched, [P, M, K] x [P, K, N]).  Its
backward materialises the transposed operand and calls ``bmm`` on contiguous tensors instead of
handing transposed views to the library: with the installed ROCm stack, the transposed-operand
bf16 batched GEMM of shape (m 2048, n 4096, k 768) -- the input gradient of the 125M LM's FFN
down projection -- returns wrong results for batches 1..P-1 (hipBLASLt reports an internal
error and the fallback path then faults).  ``scripts/check_bmm.py`` reproduces it; the NN-layout
forms are exact for every shape the LM and CNN paths use.  The extra transposes move a few MB
per GEMM.
"""
from __future__ import annotations

import torch


class _PBmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return torch.bmm(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = torch.bmm(g, b.transpose(1, 2).contiguous())
        if ctx.needs_input_grad[1]:
            db = torch.bmm(a.transpose(1, 2).contiguous(), g)
        return da, db


def pbmm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.device.type != "cuda":
        return torch.bmm(a, b)
    return _PBmm.apply(a, b)
