"""Convolution and BatchNorm operators of the population ResNet (north-star kernels K3, K8).

A 3x3 convolution (pad 1, stride 1/2) over NHWC bf16 activations with the population folded into
the batch dimension runs as HIP ``im2col`` + a population-batched GEMM (``torch.bmm`` on
hipBLASLt) ``col[P, M, 9C] . W[P, 9C, Cout]``; its backward is the GEMM's autograd plus the HIP
``col2im`` (gather form, no atomics).  BatchNorm with the residual add and ReLU fused into one
apply pass, per-trial batch statistics and running statistics, forward and backward, is HIP.

fp32 PyTorch references of both (``conv3x3_ref``, ``bn_act_ref``) are the CPU backend and the
numerics oracle of tests/test_resnet_gpu.py.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .gemm import pbmm

c_void_p, c_int, c_float, c_int64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64

_lib.register_signatures({
    "mopt_im2col": ([c_void_p, c_void_p] + [c_int] * 7 + [c_void_p], c_int),
    "mopt_col2im": ([c_void_p, c_void_p] + [c_int] * 7 + [c_void_p], c_int),
    "mopt_bn_fwd": ([c_void_p] * 8 + [c_int, c_int64, c_int, c_float, c_float, c_int, c_int,
                                     c_void_p], c_int),
    "mopt_bn_bwd": ([c_void_p] * 8 + [c_int, c_int64, c_int, c_int, c_void_p], c_int),
})


def _call(name, *args):
    lib = _lib.get_lib()
    _lib.check(getattr(lib, name)(*args), name)


def _s(t):
    return _lib.stream_ptr(t.device)


def out_hw(H, stride):
    return (H - 1) // stride + 1


# ------------------------------------------------------------------ references
def im2col_ref(x, stride):
    """x [N, H, W, C] -> col [N * OH * OW, 9 C] ((kh, kw, c) order, zero padding 1)."""
    N, H, W, C = x.shape
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1))
    OH, OW = out_hw(H, stride), out_hw(W, stride)
    taps = [xp[:, kh:kh + stride * (OH - 1) + 1:stride, kw:kw + stride * (OW - 1) + 1:stride, :]
            for kh in range(3) for kw in range(3)]
    return torch.stack(taps, 3).reshape(N * OH * OW, 9 * C)


def conv3x3_ref(x, w, P, stride):
    """x [P*B, H, W, Cin], w [P, 9 Cin, Cout] -> [P*B, OH, OW, Cout]."""
    N, H, W, C = x.shape
    OH, OW = out_hw(H, stride), out_hw(W, stride)
    col = im2col_ref(x, stride).view(P, -1, 9 * C)
    out = torch.bmm(col, w)
    return out.view(N, OH, OW, w.shape[-1])


def bn_act_ref(x, gamma, beta, running, P, train, res=None, relu=True, eps=1e-5,
               momentum=0.1):
    """x [P*B, H, W, C]; gamma/beta [P, C]; running [P, 2, C] (updated in place when train)."""
    C = x.shape[-1]
    xf = x.float().reshape(P, -1, C)
    if train:
        mean = xf.mean(1)
        var = xf.var(1, unbiased=False)
        M = xf.shape[1]
        with torch.no_grad():
            running[:, 0].mul_(1 - momentum).add_(momentum * mean.detach())
            running[:, 1].mul_(1 - momentum).add_(momentum * var.detach() * M / max(M - 1, 1))
    else:
        mean, var = running[:, 0], running[:, 1]
    y = (xf - mean[:, None]) * torch.rsqrt(var[:, None] + eps) * gamma.float()[:, None] + \
        beta.float()[:, None]
    if res is not None:
        y = y + res.float().reshape(P, -1, C)
    if relu:
        y = torch.relu(y)
    return y.reshape(x.shape).to(x.dtype)


# ------------------------------------------------------------------ HIP autograd Functions
class _Im2Col(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stride):
        N, H, W, C = x.shape
        OH, OW = out_hw(H, stride), out_hw(W, stride)
        col = torch.empty(N * OH * OW, 9 * C, dtype=x.dtype, device=x.device)
        _call("mopt_im2col", x.data_ptr(), col.data_ptr(), N, H, W, C, OH, OW, stride, _s(x))
        ctx.dims = (N, H, W, C, OH, OW, stride)
        return col

    @staticmethod
    def backward(ctx, dcol):
        N, H, W, C, OH, OW, stride = ctx.dims
        dcol = dcol.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dcol.dtype, device=dcol.device)
        _call("mopt_col2im", dcol.data_ptr(), dx.data_ptr(), N, H, W, C, OH, OW, stride,
              _s(dcol))
        return dx, None


def conv3x3(x, w, P, stride):
    """Population 3x3 convolution: x [P*B, H, W, Cin] bf16, w [P, 9 Cin, Cout]."""
    if x.device.type != "cuda":
        return conv3x3_ref(x, w, P, stride)
    N, H, W, C = x.shape
    col = _Im2Col.apply(x.contiguous(), stride)
    out = pbmm(col.view(P, -1, 9 * C), w, w.grad if w.requires_grad and w.is_leaf else None)
    return out.view(N, out_hw(H, stride), out_hw(W, stride), w.shape[-1])


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, running, P, train, relu, eps, momentum):
        C = x.shape[-1]
        M = x.numel() // (P * C)
        y = torch.empty_like(x)
        stat = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        sums = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        _call("mopt_bn_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
              0 if res is None else res.data_ptr(), y.data_ptr(), stat.data_ptr(),
              running.data_ptr(), sums.data_ptr(), P, M, C, eps, momentum, int(train), int(relu),
              _s(x))
        ctx.save_for_backward(x, y, stat, gamma)
        ctx.meta = (P, M, C, relu, res is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, stat, gamma = ctx.saved_tensors
        P, M, C, relu, has_res = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        sums = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        _call("mopt_bn_bwd", x.data_ptr(), y.data_ptr(), dy.data_ptr(), stat.data_ptr(),
              gamma.data_ptr(), dx.data_ptr(), 0 if dres is None else dres.data_ptr(),
              sums.data_ptr(), P, M, C, int(relu), _s(x))
        dgamma = sums[:, 1].to(gamma.dtype)
        dbeta = sums[:, 0].to(gamma.dtype)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


def bn_act(x, gamma, beta, running, P, train, res=None, relu=True, eps=1e-5, momentum=0.1):
    """y = relu?(BN(x) + res?) per trial; ``running`` [P, 2, C] f32 updated when training."""
    if x.device.type != "cuda":
        return bn_act_ref(x, gamma, beta, running, P, train, res, relu, eps, momentum)
    return _BNAct.apply(x.contiguous(), gamma.contiguous(), beta.contiguous(),
                        None if res is None else res.contiguous(), running, P, train, relu, eps,
                        momentum)
