"""Convolution and BatchNorm operators of the population ResNet (north-star kernels K3, K8).

A 3x3 convolution (pad 1, stride 1/2) over NHWC bf16 activations with the population folded into
the batch dimension is an implicit GEMM on the population MFMA kernel (``csrc/pgemm.hip``,
``mopt_pconv``): the forward ``y = im2col(x) . W``, the input gradient (the transposed
convolution ``dx = gather(dy) . W'``) and the weight gradient ``dW = im2col(x)^T . dy`` (split-K
over pixels) gather their operands straight from the NHWC tensors, so no im2col / col2im matrix
(9x the activation) is ever written to HBM; the weight gradient lands directly in the flat
gradient buffer of the fused optimizer.  BatchNorm with the residual add and ReLU fused into one
apply pass, per-trial batch statistics and running statistics, forward and backward, is HIP.

fp32 PyTorch references of both (``conv3x3_ref``, ``bn_act_ref``) are the CPU backend and the
numerics oracle of tests/test_resnet_gpu.py.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from .gemm import plan

c_void_p, c_int, c_float, c_int64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64

_lib.register_signatures({
    "mopt_bn_fwd": ([c_void_p] * 8 + [c_int, c_int64, c_int, c_float, c_float, c_int, c_int,
                                     c_int, c_int, c_int, c_void_p], c_int),
    "mopt_bn_bwd": ([c_void_p] * 11 + [c_int, c_int64, c_int, c_int, c_int, c_void_p], c_int),
    "mopt_pconv": ([c_int] + [c_void_p] * 4 + [c_int] * 10 + [c_void_p], c_int),
    "mopt_dconv": ([c_int] + [c_void_p] * 4 + [c_int] * 7 + [c_void_p], c_int),
    "mopt_dconv_wgrad_splits": ([c_int] * 6, c_int),
    "mopt_dconv_shared_x": ([c_int] + [c_void_p] * 4 + [c_int] * 6 + [c_void_p], c_int),
    "mopt_dconv_bnin": ([c_int] + [c_void_p] * 4 + [c_int] * 5 + [c_void_p] * 5 +
                        [c_int64, c_float, c_float, c_void_p], c_int),
    "mopt_dconv_dgrad_bnsums": ([c_void_p] * 4 + [c_int] * 5 + [c_void_p] * 5, c_int),
    "mopt_dconv_dgrad_bnres": ([c_void_p] * 5 + [c_int] * 7 + [c_void_p] * 4, c_int),
    "mopt_dconv_bnres_fwd": ([c_void_p] * 6 + [c_int] + [c_void_p] * 3 + [c_int] * 6 +
                             [c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p], c_int),
    "mopt_resnet_head_bn": ([c_void_p] * 8 + [c_int] * 5 + [c_float] + [c_void_p] * 9 +
                            [c_int64, c_float, c_float, c_void_p], c_int),
    "mopt_resnet_head": ([c_void_p] * 4 + [c_int] * 5 + [c_float, c_int] + [c_void_p] * 7,
                         c_int),
    "mopt_resnet_head_part_floats": ([c_int] * 3, c_int),
})
# BatchNorm 1 + ReLU applied while conv 2 stages its input (6.71 -> 6.55 ms/step, round 3); the
# materialised path remains for evaluation and shapes the fused kernels do not take
_BN_INTO_CONV = True
# the backward of a block output's BatchNorm (relu(BN(x) + shortcut)) fused into the data
# gradient of the next block's first convolution (``_bn_res_dgrad``; MOPT_BN_RES_DGRAD=0: the
# separate reduce + apply passes, for A/B runs)
_BN_RES_DGRAD = os.environ.get("MOPT_BN_RES_DGRAD", "1") != "0"
# ... and its forward apply pass folded into that convolution's input staging (``PendingBN``,
# ``bn_res_conv3x3``; MOPT_BN_RES_FWD=0: the separate apply pass)
_BN_RES_FWD = os.environ.get("MOPT_BN_RES_FWD", "1") != "0"
# the BatchNorms whose apply runs inside a convolution's staging are also finalized there (the
# kernel derives mean / rstd from the batch sums, its trial's first workgroup stores them and
# the running update): no bn_finalize launch (MOPT_BN_FIN_IN_CONV=0: the separate launch)
_BN_FIN_IN_CONV = os.environ.get("MOPT_BN_FIN_IN_CONV", "1") != "0"
# (Ci, Co, stride) of the direct forward with the block output formed in its staging
# (csrc/conv_direct.hip mopt_dconv_bnres_fwd): shortcut shaped like x or none / option-A
_BNRES_FWD_SHAPES = {(16, 16, 1), (16, 32, 2), (32, 32, 1), (32, 64, 2), (64, 64, 1)}
_BNRES_FWD_SHAPES_SUB2 = {(32, 32, 1), (64, 64, 1)}

_NOT_SUPPORTED = 801   # hipErrorNotSupported: no direct-conv instantiation for the shape
# direct convolution kernels for square inputs; the implicit GEMM (pgemm gathers) is the
# fallback for the rest (scripts/conv_bench.py flips this to compare the two)
_DIRECT = True


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
def _pow2(v):
    return v >= 1 and (v & (v - 1)) == 0


def _dconv(kind, a, b, out, P, Bn, H, W, Ci, Co, stride, sums=None, addend=None, addend_c=0):
    """Direct (halo-tiled) convolution kernels of csrc/conv_direct.hip; False when the shape has
    no instantiation (the caller then runs the implicit GEMM)."""
    if not _DIRECT or H != W:
        return False
    lib = _lib.get_lib()
    aux = sums if kind == 0 else addend
    if kind == 2:
        nb = lib.mopt_dconv_wgrad_splits(P, Bn, H, Ci, Co, stride)
        if nb <= 0:
            return False
        aux = torch.empty(nb * P * 9 * Ci * Co, dtype=torch.float32, device=out.device)
    rc = lib.mopt_dconv(kind, a.data_ptr(), b.data_ptr(), out.data_ptr(),
                        0 if aux is None else aux.data_ptr(), P, Bn, H, Ci, Co, stride,
                        addend_c if kind == 1 else 0, _s(out))
    if rc == _NOT_SUPPORTED:
        return False
    _lib.check(rc, "mopt_dconv")
    return True


def _pconv(kind, a, b, out, P, Bn, H, W, Ci, Co, stride, sums=None, addend=None, addend_c=0):
    """``addend`` (kind 1): added to the data gradient -- shaped like ``out``, or (``addend_c``
    > 0) the half-resolution gradient of an option-A shortcut, added at the even pixels."""
    if _dconv(kind, a, b, out, P, Bn, H, W, Ci, Co, stride, sums, addend, addend_c):
        return out, sums is not None
    OH, OW = out_hw(H, stride), out_hw(W, stride)
    M, N, K = {0: (Bn * OH * OW, Co, 9 * Ci), 1: (Bn * H * W, Ci, 9 * Co),
               2: (9 * Ci, Co, Bn * OH * OW)}[kind]
    cfg, splits, kps = plan(P, M, N, K)
    if kind != 2:
        splits, kps = 1, K
    part = (torch.empty(splits, P, M, N, dtype=torch.float32, device=out.device)
            if splits > 1 else None)
    _call("mopt_pconv", kind, a.data_ptr(), b.data_ptr(), out.data_ptr(),
          0 if part is None else part.data_ptr(), P, Bn, H, W, Ci, Co, stride, cfg, splits, kps,
          _s(out))
    if addend is not None and addend_c:
        out[:, ::2, ::2, :] += addend[..., :out.shape[-1]]
    elif addend is not None:
        out.add_(addend)
    return out, False


def _bn_res_dgrad(dy, w, dx, addend, sub2, link, P, Bn, H, W, Ci, Co, stride) -> bool:
    """Data gradient of a convolution whose input is the output of a linked BatchNorm (``link``,
    filled by ``_BNAct.forward``: relu(BN(x) + shortcut) of the previous block, or the stem's
    relu(BN(x))): dx = (dgrad(dy) + addend) relu'(link y), the gradient behind that ReLU, and the
    BatchNorm backward's reductions added into its zeroed ``link["sums"]``
    (csrc/conv_direct.hip ``mopt_dconv_dgrad_bnres``).  False when the shape has no kernel: the
    caller runs the plain data gradient and the BatchNorm its own reduction."""
    if not (_BN_RES_DGRAD and _DIRECT and H == W and addend is not None):
        return False
    if (stride == 2) != bool(sub2):
        return False
    rc = _lib.get_lib().mopt_dconv_dgrad_bnres(
        dy.data_ptr(), w.data_ptr(), dx.data_ptr(), addend.data_ptr(), link["sums"].data_ptr(),
        P, Bn, H, Ci, Co, stride, addend.shape[-1] if sub2 else 0, link["x"].data_ptr(),
        link["y"].data_ptr(), link["stat"].data_ptr(), _s(dx))
    if rc == _NOT_SUPPORTED:
        return False
    _lib.check(rc, "mopt_dconv_dgrad_bnres")
    return True


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, P, stride, grad_out, stats=None, mailbox=None, bn_link=None):
        N, H, W, Ci = x.shape
        Co = w.shape[-1]
        Bn = N // P
        y = torch.empty(N, out_hw(H, stride), out_hw(W, stride), Co, dtype=x.dtype,
                        device=x.device)
        # stats = [zeroed f32 sums [P, 2, Co], False]: the direct kernel adds the BatchNorm
        # batch sums of y and sets the flag
        _, done = _pconv(0, x, w, y, P, Bn, H, W, Ci, Co, stride,
                         None if stats is None else stats[0])
        if stats is not None:
            stats[1] = done
        ctx.save_for_backward(x, w)
        ctx.meta = (P, Bn, H, W, Ci, Co, stride)
        ctx.grad_out = grad_out
        ctx.mailbox = mailbox
        ctx.bn_link = bn_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        P, Bn, H, W, Ci, Co, stride = ctx.meta
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            # the identity shortcut's gradient (left by the block's last BatchNorm) joins here,
            # in the data-gradient epilogue, instead of in a separate autograd add
            addend = ctx.mailbox.pop("dres", None) if ctx.mailbox is not None else None
            sub2 = addend is not None and ctx.mailbox.pop("sub2", False)
            link = ctx.bn_link
            if link is not None and _bn_res_dgrad(dy, w, dx, addend, sub2, link, P, Bn, H, W,
                                                  Ci, Co, stride):
                link["fused"] = True     # dx is dz, its BatchNorm's reductions are summed
            else:
                _pconv(1, dy, w, dx, P, Bn, H, W, Ci, Co, stride, addend=addend,
                       addend_c=addend.shape[-1] if sub2 else 0)
        if ctx.needs_input_grad[1]:
            if ctx.grad_out is not None:         # straight into the flat gradient buffer
                _pconv(2, x, dy, ctx.grad_out, P, Bn, H, W, Ci, Co, stride)
            else:
                dw = torch.empty_like(w)
                _pconv(2, x, dy, dw, P, Bn, H, W, Ci, Co, stride)
        return dx, dw, None, None, None, None, None, None


def conv3x3(x, w, P, stride, stats=None, mailbox=None, bn_link=None):
    """Population 3x3 convolution: x [P*B, H, W, Cin] bf16, w [P, 9 Cin, Cout].  ``stats`` (HIP
    only): ``[sums, False]`` with zeroed f32 sums [P, 2, Cout]; when the direct kernel ran, the
    per-trial channel sums of the output and of its square were added and the flag is True."""
    if x.device.type != "cuda":
        return conv3x3_ref(x, w, P, stride)
    N, H, W, C = x.shape
    Co = w.shape[-1]
    if N % P or not all(_pow2(v) for v in (H, W, C, Co)) or C < 8 or Co < 8 or \
            tuple(w.shape) != (P, 9 * C, Co):
        raise ValueError(f"conv3x3: needs power-of-two H, W, channels (>= 8) and w [P, 9C, Co]; "
                         f"got x {tuple(x.shape)} w {tuple(w.shape)} P {P}")
    grad_out = w.grad if (w.requires_grad and w.is_leaf and w.grad is not None) else None
    return _Conv3x3.apply(x.contiguous(), w.contiguous(), P, stride, grad_out, stats, mailbox,
                          bn_link)


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, running, P, train, relu, eps, momentum, sums=None,
                arena=None, mailbox=None, res_sub2=False, link=None):
        C = x.shape[-1]
        M = x.numel() // (P * C)
        y = torch.empty_like(x)
        stat = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        ready = sums is not None and train
        if not ready:
            sums = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        _call("mopt_bn_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
              0 if res is None else res.data_ptr(), y.data_ptr(), stat.data_ptr(),
              running.data_ptr(), sums.data_ptr(), P, M, C, eps, momentum, int(train), int(relu),
              int(ready), res.shape[-1] if res_sub2 else 0,
              (x.shape[1].bit_length() - 1) if res_sub2 else 0, _s(x))
        ctx.save_for_backward(x, y, stat, gamma, beta)
        ctx.meta = (P, M, C, relu, res is not None)
        # backward: pre-zeroed sums from the step's arena; dgamma / dbeta written by the kernel
        # straight into the flat gradient buffer when the parameters are its leaf views
        ctx.bwd_sums = arena.take(P * 2 * C).view(P, 2, C) if arena is not None else None
        ctx.grads = tuple(t.grad if (t.requires_grad and t.is_leaf and t.grad is not None) else None
                          for t in (gamma, beta))
        ctx.mailbox = mailbox
        ctx.res_sub2 = res_sub2
        # link: the consumer convolution's data gradient may do this backward's masking and
        # reductions (_bn_res_dgrad) -- it needs the zeroed backward sums, x, y and the statistics
        ctx.link = None
        if link is not None and train and relu and ctx.bwd_sums is not None:
            link.update(x=x, y=y, stat=stat, sums=ctx.bwd_sums, fused=False)
            ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, stat, gamma, beta = ctx.saved_tensors
        P, M, C, relu, has_res = ctx.meta
        if ctx.link is not None and ctx.link.pop("fused", False):
            return _BNAct._fused_backward(ctx, dy, x, stat, gamma, beta, P, M, C, has_res)
        # without a residual relu'(.) is recomputed from x, gamma, beta (y is not read): one
        # activation tensor less through both backward kernels
        mode = 0 if not relu else (1 if has_res else 2)
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        zeroed = ctx.bwd_sums is not None
        sums = ctx.bwd_sums if zeroed else torch.empty(P, 2, C, dtype=torch.float32,
                                                       device=x.device)
        gg, gb = ctx.grads
        direct = gg is not None and gb is not None and gg.is_contiguous() and gb.is_contiguous()
        _call("mopt_bn_bwd", x.data_ptr(), y.data_ptr(), dy.data_ptr(), stat.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), dx.data_ptr(),
              0 if dres is None else dres.data_ptr(), sums.data_ptr(),
              gg.data_ptr() if direct else 0, gb.data_ptr() if direct else 0,
              P, M, C, mode, int(zeroed), _s(x))
        if dres is not None and ctx.mailbox is not None:
            ctx.mailbox["dres"] = dres     # picked up by the block's first convolution
            ctx.mailbox["sub2"] = ctx.res_sub2
            dres = None
        if direct:
            return dx, None, None, dres, None, None, None, None, None, None, None, None, None, \
                None, None
        dgamma = sums[:, 1].to(gamma.dtype)
        dbeta = sums[:, 0].to(gamma.dtype)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, \
            None, None

    @staticmethod
    def _fused_backward(ctx, dz, x, stat, gamma, beta, P, M, C, has_res):
        """Backward after the consumer's data gradient (``_bn_res_dgrad``) delivered dz (the
        gradient behind the ReLU) and summed its reductions: the apply pass alone, no mask, and
        dz itself is the shortcut's gradient (no copy written)."""
        ctx.link.clear()
        dz = dz.contiguous()
        dx = torch.empty_like(x)
        gg, gb = ctx.grads
        direct = gg is not None and gb is not None and gg.is_contiguous() and gb.is_contiguous()
        _call("mopt_bn_bwd", x.data_ptr(), 0, dz.data_ptr(), stat.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), dx.data_ptr(), 0, ctx.bwd_sums.data_ptr(),
              gg.data_ptr() if direct else 0, gb.data_ptr() if direct else 0, P, M, C, 0, 2, _s(x))
        dres = dz if has_res else None
        if dres is not None and ctx.mailbox is not None:
            ctx.mailbox["dres"] = dres
            ctx.mailbox["sub2"] = ctx.res_sub2
            dres = None
        dgamma = dbeta = None
        if not direct:
            dgamma = ctx.bwd_sums[:, 1].to(gamma.dtype)
            dbeta = ctx.bwd_sums[:, 0].to(gamma.dtype)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, \
            None


class _BNReluConv3x3(torch.autograd.Function):
    """``conv3x3(relu(BN(x)), w)`` of a stride-1 convolution over a training-mode BatchNorm
    whose output has no other consumer (the second convolution of a ResNet basic block): the
    BatchNorm computes its statistics only (batch sums from the producing convolution's
    epilogue) and the convolution applies ``relu(x sc + sh)`` while staging its halo bands, in
    the forward and again in the weight gradient -- the BatchNorm output (one activation tensor
    written and read back per layer) never reaches HBM.  Backward: data gradient of the
    convolution, the BatchNorm backward with relu' recomputed from x (mode 2), weight gradient
    with the BatchNorm re-applied on the fly."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w, running, P, eps, momentum, sums, out_sums, arena,
                grad_w):
        N, H, W, C = x.shape
        Co = w.shape[-1]
        M = x.numel() // (P * C)
        stat = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        fin = _BN_FIN_IN_CONV
        if not fin:
            _call("mopt_bn_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 0, 0,
                  stat.data_ptr(), running.data_ptr(), sums.data_ptr(), P, M, C, eps, momentum,
                  1, 1, 1, 0, 0, _s(x))
        y = torch.empty(N, H, W, Co, dtype=x.dtype, device=x.device)
        _call("mopt_dconv_bnin", 0, x.data_ptr(), w.data_ptr(), y.data_ptr(),
              out_sums.data_ptr(), P, N // P, H, C, Co, stat.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), sums.data_ptr() if fin else 0, running.data_ptr() if fin else 0,
              M, eps, momentum, _s(x))
        ctx.save_for_backward(x, gamma, beta, w, stat)
        ctx.meta = (P, M, C, Co)
        ctx.bwd_sums = arena.take(P * 2 * C).view(P, 2, C) if arena is not None else None
        ctx.grads = tuple(t.grad if (t.requires_grad and t.is_leaf and t.grad is not None) else None
                          for t in (gamma, beta))
        ctx.grad_w = grad_w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, w, stat = ctx.saved_tensors
        P, M, C, Co = ctx.meta
        N, H, W, _ = x.shape
        Bn = N // P
        dy = dy.contiguous()
        # data gradient of the convolution = the BatchNorm output's gradient; its epilogue also
        # accumulates the BatchNorm backward's reductions into the zeroed sums (flag 2: the
        # BatchNorm backward then runs its apply pass only)
        dbn = torch.empty_like(x)
        sums = ctx.bwd_sums if ctx.bwd_sums is not None else \
            torch.zeros(P, 2, C, dtype=torch.float32, device=x.device)
        rc = _lib.get_lib().mopt_dconv_dgrad_bnsums(
            dy.data_ptr(), w.data_ptr(), dbn.data_ptr(), sums.data_ptr(), P, Bn, H, C, Co,
            x.data_ptr(), stat.data_ptr(), gamma.data_ptr(), beta.data_ptr(), _s(x))
        if rc == _NOT_SUPPORTED:
            _pconv(1, dy, w, dbn, P, Bn, H, W, C, Co, 1)
            zeroed = 1
        else:
            _lib.check(rc, "mopt_dconv_dgrad_bnsums")
            zeroed = 2
        dx = torch.empty_like(x)
        gg, gb = ctx.grads
        direct = gg is not None and gb is not None and gg.is_contiguous() and gb.is_contiguous()
        _call("mopt_bn_bwd", x.data_ptr(), 0, dbn.data_ptr(), stat.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), dx.data_ptr(), 0, sums.data_ptr(),
              gg.data_ptr() if direct else 0, gb.data_ptr() if direct else 0,
              P, M, C, 2, zeroed, _s(x))
        # weight gradient over relu(BN(x)), applied again while staging
        dw = ctx.grad_w if ctx.grad_w is not None else torch.empty_like(w)
        lib = _lib.get_lib()
        nb = lib.mopt_dconv_wgrad_splits(P, Bn, H, C, Co, 1)
        part = torch.empty(max(nb, 1) * P * 9 * C * Co, dtype=torch.float32, device=x.device)
        _call("mopt_dconv_bnin", 2, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), part.data_ptr(),
              P, Bn, H, C, Co, stat.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 0, 0, 0, 0.0,
              0.0, _s(x))
        dgamma = dbeta = None
        if not direct:
            dgamma = sums[:, 1].to(gamma.dtype)
            dbeta = sums[:, 0].to(gamma.dtype)
        return (dx, dgamma, dbeta, None if ctx.grad_w is not None else dw) + (None,) * 8


def bn_into_conv_ok(x, w, P, stride, train, arena, sums_ready) -> bool:
    """Whether ``bn_relu_conv3x3`` can run: training with the step's zero arena and the batch
    sums of x from its producing convolution, a stride-1 square convolution with Ci == Co in
    {16, 32, 64} on the direct kernels."""
    if not (_BN_INTO_CONV and _DIRECT and train and arena is not None and sums_ready):
        return False
    if x.device.type != "cuda" or stride != 1:
        return False
    N, H, W, C = x.shape
    return H == W and _pow2(H) and C in (16, 32, 64) and tuple(w.shape) == (P, 9 * C, C) and \
        N % P == 0 and _lib.get_lib().mopt_dconv_wgrad_splits(P, N // P, H, C, C, 1) > 0


def bn_relu_conv3x3(x, gamma, beta, running, w, P, sums, arena, eps=1e-5, momentum=0.1):
    """``(conv3x3(relu(BN(x)), w), batch sums of that output)`` with the BatchNorm applied inside
    the convolution (``_BNReluConv3x3``); ``sums``: x's batch sums from its producing
    convolution.  Check ``bn_into_conv_ok`` first."""
    Co = w.shape[-1]
    out_sums = arena.take(P * 2 * Co).view(P, 2, Co)
    grad_w = w.grad if (w.requires_grad and w.is_leaf and w.grad is not None) else None
    y = _BNReluConv3x3.apply(x.contiguous(), gamma.contiguous(), beta.contiguous(),
                             w.contiguous(), running, P, eps, momentum, sums, out_sums, arena,
                             grad_w)
    return y, out_sums


class PendingBN:
    """A training ``relu(BN(x) + shortcut?)`` whose apply pass has not run yet: x with its batch
    sums (from the producing convolution's epilogue), the BatchNorm's parameters, the shortcut
    (``res``: shaped like x, or with ``res_sub2`` the full-resolution block input of an option-A
    shortcut; None for the stem) and the block's mailbox (the shortcut gradient goes there).  The
    consumer convolution forms the output in its input staging (``bn_res_conv3x3``) or calls
    ``materialize``."""

    __slots__ = ("x", "sums", "gamma", "beta", "running", "res", "res_sub2", "mailbox", "P")

    def __init__(self, x, sums, gamma, beta, running, P, res=None, res_sub2=False, mailbox=None):
        self.x, self.sums, self.gamma, self.beta, self.running = x, sums, gamma, beta, running
        self.res, self.res_sub2, self.mailbox, self.P = res, res_sub2, mailbox, P

    def materialize(self, arena, link=None):
        return bn_act(self.x, self.gamma, self.beta, self.running, self.P, True, res=self.res,
                      sums=self.sums, arena=arena, mailbox=self.mailbox, res_sub2=self.res_sub2,
                      link=link)


def bn_res_conv_ok(pend: PendingBN, w, stride) -> bool:
    """Whether ``bn_res_conv3x3`` has a kernel for this block output and convolution."""
    if not (_BN_RES_FWD and _DIRECT) or pend is None or pend.sums is None:
        return False
    x = pend.x
    if x.device.type != "cuda":
        return False
    N, H, W, C = x.shape
    Co = w.shape[-1]
    if H != W or not _pow2(H) or N % pend.P or tuple(w.shape) != (pend.P, 9 * C, Co):
        return False
    if pend.res is not None and pend.res_sub2:
        r = pend.res
        return (C, Co, stride) in _BNRES_FWD_SHAPES_SUB2 and r.shape[0] == N and \
            tuple(r.shape[1:3]) == (2 * H, 2 * H) and r.shape[-1] % 8 == 0 and r.shape[-1] <= C
    if pend.res is not None and tuple(pend.res.shape) != tuple(x.shape):
        return False
    return (C, Co, stride) in _BNRES_FWD_SHAPES


class _BNResConv3x3(torch.autograd.Function):
    """``conv3x3(relu(BN(x) + shortcut), w)`` and the block output itself, for a training
    BatchNorm whose output feeds this convolution (the first of the next basic block): the
    BatchNorm computes its statistics only, the convolution forms the block output while staging
    its input bands and writes it to HBM once (it is the next shortcut, the relu' mask of the
    backward and this convolution's weight-gradient operand) -- the separate apply pass is gone.
    Backward: the data gradient with the BatchNorm's masking and reductions in its epilogue
    (``_bn_res_dgrad``), the BatchNorm's apply pass, dz as the block's shortcut gradient, the
    weight gradient over the stored block output."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w, res, running, P, stride, sums, out_sums, arena,
                bn_mailbox, res_sub2, conv_mailbox, grad_w, eps, momentum):
        N, H, W, C = x.shape
        Co = w.shape[-1]
        M = x.numel() // (P * C)
        stat = torch.empty(P, 2, C, dtype=torch.float32, device=x.device)
        fin = _BN_FIN_IN_CONV
        if not fin:
            _call("mopt_bn_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 0, 0,
                  stat.data_ptr(), running.data_ptr(), sums.data_ptr(), P, M, C, eps, momentum,
                  1, 1, 1, 0, 0, _s(x))
        h = torch.empty_like(x)
        OH = out_hw(H, stride)
        y = torch.empty(N, OH, OH, Co, dtype=x.dtype, device=x.device)
        res_c = res.shape[-1] if (res is not None and res_sub2) else 0
        _call("mopt_dconv_bnres_fwd", x.data_ptr(), w.data_ptr(), y.data_ptr(),
              out_sums.data_ptr(), h.data_ptr(), 0 if res is None else res.data_ptr(), res_c,
              stat.data_ptr(), gamma.data_ptr(), beta.data_ptr(), P, N // P, H, C, Co, stride,
              sums.data_ptr() if fin else 0, running.data_ptr() if fin else 0, M, eps, momentum,
              _s(x))
        ctx.save_for_backward(x, h, stat, gamma, beta, w)
        ctx.meta = (P, N // P, H, C, Co, stride, M)
        ctx.bwd_sums = arena.take(P * 2 * C).view(P, 2, C)
        ctx.grads = tuple(t.grad if (t.requires_grad and t.is_leaf and t.grad is not None) else None
                          for t in (gamma, beta))
        ctx.bn_mailbox, ctx.res_sub2, ctx.has_res = bn_mailbox, res_sub2, res is not None
        ctx.conv_mailbox, ctx.grad_w = conv_mailbox, grad_w
        ctx.mark_non_differentiable(h)
        # (h has no gradient: without this autograd hands backward a zero-filled dh -- a 134 MB
        #  fill per stage-1 block, measured +120 us per ResNet-20 step)
        ctx.set_materialize_grads(False)
        return y, h

    @staticmethod
    def backward(ctx, dy, dh):
        x, h, stat, gamma, beta, w = ctx.saved_tensors
        P, Bn, H, C, Co, stride, M = ctx.meta
        dy = dy.contiguous()
        box = ctx.conv_mailbox
        addend = box.pop("dres", None) if box is not None else None
        sub2 = addend is not None and box.pop("sub2", False)
        g = torch.empty_like(x)
        link = {"x": x, "y": h, "stat": stat, "sums": ctx.bwd_sums}
        if _bn_res_dgrad(dy, w, g, addend, sub2, link, P, Bn, H, H, C, Co, stride):
            mode, zeroed = 0, 2          # g = dz (masked), its reductions summed
        else:
            _pconv(1, dy, w, g, P, Bn, H, H, C, Co, stride, addend=addend,
                   addend_c=addend.shape[-1] if sub2 else 0)
            mode, zeroed = 1, 1          # g = the block output's gradient: mask from h
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if (mode == 1 and ctx.has_res) else None
        gg, gb = ctx.grads
        direct = gg is not None and gb is not None and gg.is_contiguous() and gb.is_contiguous()
        _call("mopt_bn_bwd", x.data_ptr(), h.data_ptr(), g.data_ptr(), stat.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), dx.data_ptr(),
              0 if dres is None else dres.data_ptr(), ctx.bwd_sums.data_ptr(),
              gg.data_ptr() if direct else 0, gb.data_ptr() if direct else 0, P, M, C, mode,
              zeroed, _s(x))
        if ctx.has_res and ctx.bn_mailbox is not None:
            ctx.bn_mailbox["dres"] = g if mode == 0 else dres
            ctx.bn_mailbox["sub2"] = ctx.res_sub2
        dw = ctx.grad_w if ctx.grad_w is not None else torch.empty_like(w)
        _pconv(2, h, dy, dw, P, Bn, H, H, C, Co, stride)
        dgamma = dbeta = None
        if not direct:
            dgamma = ctx.bwd_sums[:, 1].to(gamma.dtype)
            dbeta = ctx.bwd_sums[:, 0].to(gamma.dtype)
        return (dx, dgamma, dbeta, None if ctx.grad_w is not None else dw) + (None,) * 13


def bn_res_conv3x3(pend: PendingBN, w, P, stride, arena, conv_mailbox=None, eps=1e-5,
                   momentum=0.1):
    """``(conv3x3(h, w), batch sums of that output, h)`` with h = relu(BN(x) + shortcut) of the
    pending BatchNorm formed inside the convolution (``_BNResConv3x3``); check
    ``bn_res_conv_ok`` first.  ``conv_mailbox``: this convolution's block mailbox (the block's
    shortcut gradient arrives there)."""
    Co = w.shape[-1]
    out_sums = arena.take(P * 2 * Co).view(P, 2, Co)
    grad_w = w.grad if (w.requires_grad and w.is_leaf and w.grad is not None) else None
    res = None if pend.res is None else pend.res.detach().contiguous()
    y, h = _BNResConv3x3.apply(pend.x.contiguous(), pend.gamma.contiguous(),
                               pend.beta.contiguous(), w.contiguous(), res, pend.running, P,
                               stride, pend.sums, out_sums, arena, pend.mailbox, pend.res_sub2,
                               conv_mailbox, grad_w, eps, momentum)
    return y, out_sums, h


class _SharedInputConv3x3(torch.autograd.Function):
    """The stem: a stride-1 convolution of the minibatch every trial shares, x [Bn, H, W, Ci]
    (no P-fold copy), with the output's BatchNorm batch sums; backward: the weight gradient only
    (the input needs none)."""

    @staticmethod
    def forward(ctx, x, w, P, sums, grad_out):
        Bn, H, W, Ci = x.shape
        Co = w.shape[-1]
        y = torch.empty(P * Bn, H, W, Co, dtype=x.dtype, device=x.device)
        _call("mopt_dconv_shared_x", 0, x.data_ptr(), w.data_ptr(), y.data_ptr(), sums.data_ptr(),
              P, Bn, H, Ci, Co, 1, _s(x))
        ctx.save_for_backward(x, w)
        ctx.meta = (P, Bn, H, Ci, Co)
        ctx.grad_out = grad_out
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        P, Bn, H, Ci, Co = ctx.meta
        dy = dy.contiguous()
        lib = _lib.get_lib()
        nb = lib.mopt_dconv_wgrad_splits(P, Bn, H, Ci, Co, 1)
        part = torch.empty(max(nb, 1) * P * 9 * Ci * Co, dtype=torch.float32, device=dy.device)
        dw = ctx.grad_out if ctx.grad_out is not None else torch.empty_like(w)
        _call("mopt_dconv_shared_x", 2, x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
              part.data_ptr(), P, Bn, H, Ci, Co, 1, _s(dy))
        return None, (None if ctx.grad_out is not None else dw), None, None, None


# the stem reads the shared minibatch in place (MOPT_SHARED_STEM=0: a P-fold expanded copy)
_SHARED_STEM = os.environ.get("MOPT_SHARED_STEM", "1") != "0"


def shared_conv_stats(x, w, P, arena):
    """``(conv3x3 of the shared batch x [Bn, H, W, Ci] for every trial, batch sums)`` on the HIP
    path (``_SharedInputConv3x3``), or None when the shape has no kernel / it is switched off."""
    Bn, H, W, Ci = x.shape
    Co = w.shape[-1]
    if not (_SHARED_STEM and _DIRECT) or H != W or (Ci, Co) not in ((8, 16), (16, 16)) or \
            tuple(w.shape) != (P, 9 * Ci, Co) or \
            _lib.get_lib().mopt_dconv_wgrad_splits(P, Bn, H, Ci, Co, 1) <= 0:
        return None
    sums = arena.take(P * 2 * Co).view(P, 2, Co)
    grad_out = w.grad if (w.requires_grad and w.is_leaf and w.grad is not None) else None
    y = _SharedInputConv3x3.apply(x.contiguous(), w.contiguous(), P, sums, grad_out)
    return y, sums


def conv_stats(x, w, P, stride, train, arena=None, mailbox=None, bn_link=None):
    """``(conv3x3(x, w), batch sums of the output or None)``: the first half of ``conv_bn_act``
    (HIP path; the sums come from the direct kernel's epilogue when it ran).  ``bn_link``: the
    link dict of the BatchNorm that produced x (``bn_act(link=...)``), whose backward this
    convolution's data gradient then fuses (``_bn_res_dgrad``)."""
    Co = w.shape[-1]
    stats = None
    if train:
        z = arena.take(P * 2 * Co).view(P, 2, Co) if arena is not None else \
            torch.zeros(P, 2, Co, dtype=torch.float32, device=x.device)
        stats = [z, False]
    y = conv3x3(x, w, P, stride, stats, mailbox=mailbox, bn_link=bn_link)
    return y, (stats[0] if stats is not None and stats[1] else None)


def option_a_shortcut(h, cout):
    """ResNet option-A shortcut: stride-2 subsample, zero-pad channels to ``cout`` (NHWC)."""
    y = h[:, ::2, ::2, :]
    return torch.nn.functional.pad(y, (0, cout - h.shape[-1])).contiguous()


def bn_act(x, gamma, beta, running, P, train, res=None, relu=True, eps=1e-5, momentum=0.1,
           sums=None, arena=None, mailbox=None, res_sub2=False, link=None):
    """``res_sub2``: ``res`` is the full-resolution block input and the residual its option-A
    shortcut, read in place by the kernel (no subsampled / padded copy).  ``link`` (a dict,
    training with ``arena``): filled for the consumer convolution (``conv_stats(bn_link=...)``),
    whose data gradient may take over this BatchNorm's relu' masking and reductions."""
    """y = relu?(BN(x) + res?) per trial; ``running`` [P, 2, C] f32 updated when training.
    ``sums``: precomputed f32 [P, 2, C] batch sums of x and x^2 (the producing convolution's
    epilogue) -- the statistics pass is skipped."""
    if x.device.type != "cuda" or (res_sub2 and x.shape[1] & (x.shape[1] - 1)):
        if res_sub2:
            res = option_a_shortcut(res, x.shape[-1])
        if x.device.type != "cuda":
            return bn_act_ref(x, gamma, beta, running, P, train, res, relu, eps, momentum)
        res_sub2 = False
    return _BNAct.apply(x.contiguous(), gamma.contiguous(), beta.contiguous(),
                        None if res is None else res.contiguous(), running, P, train, relu, eps,
                        momentum, sums, arena, mailbox, res_sub2, link)


class ZeroArena:
    """One zero-filled f32 buffer per training step, carved into the convolutions' BatchNorm
    sums and the BatchNorm backward's reductions (one fill instead of one per layer)."""

    def __init__(self, n, device):
        self.buf = torch.zeros(n, dtype=torch.float32, device=device)
        self.pos = 0

    def take(self, n):
        if self.pos + n > self.buf.numel():
            raise RuntimeError("ZeroArena exhausted")
        v = self.buf[self.pos:self.pos + n]
        self.pos += n
        return v


def conv_bn_act(x, w, gamma, beta, running, P, stride, train, res=None, relu=True, arena=None,
                conv_mailbox=None, bn_mailbox=None, res_sub2=False, link=None):
    """``bn_mailbox`` / ``conv_mailbox`` (one dict per residual block, HIP path): the block's last
    BatchNorm leaves the identity shortcut's gradient there and the block's first convolution
    adds it in its data-gradient epilogue -- pass ``res`` detached so autograd does not add it
    a second time."""
    """relu?(BN(conv3x3(x, w)) + res?): on the HIP path the convolution's epilogue produces the
    BatchNorm batch statistics (no separate reduction pass over the conv output)."""
    if x.device.type != "cuda":
        if res_sub2:
            res = option_a_shortcut(res, w.shape[-1])
        return bn_act_ref(conv3x3_ref(x, w, P, stride), gamma, beta, running, P, train, res,
                          relu)
    Co = w.shape[-1]
    stats = None
    if train:
        z = arena.take(P * 2 * Co).view(P, 2, Co) if arena is not None else \
            torch.zeros(P, 2, Co, dtype=torch.float32, device=x.device)
        stats = [z, False]
    y = conv3x3(x, w, P, stride, stats, mailbox=conv_mailbox)
    return bn_act(y, gamma, beta, running, P, train, res=res, relu=relu,
                  sums=stats[0] if stats is not None and stats[1] else None,
                  arena=arena if train else None, mailbox=bn_mailbox, res_sub2=res_sub2,
                  link=link)


# ------------------------------------------------------------------ classifier head
def head_ref(h, fcw, fcb, labels, P, ncls):
    """fp32 reference of the head: global average pool -> linear -> softmax cross-entropy.
    h [P*B, H, W, C] -> (per-trial loss sums [P], #correct [P], logits [P, B, ncls])."""
    B = h.shape[0] // P
    feat = h.view(P, B, -1, h.shape[-1]).float().mean(2)                    # [P, B, C]
    logits = torch.baddbmm(fcb.float()[:, None, :], feat, fcw.float())[..., :ncls]
    lab = labels.view(P, B).long()
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, ncls), lab.reshape(-1),
                                             reduction="none").view(P, B).sum(1)
    correct = (logits.argmax(-1) == lab).float().sum(1)
    return loss, correct, logits


class _Head(torch.autograd.Function):
    """Fused pool + linear + cross-entropy (csrc/resnet_head.hip).  The forward computes the
    gradients too (``scale`` = d loss_sum / d per-sample loss, e.g. 1 / B): dW and db go straight
    into the flat gradient buffer (``gw``, ``gb``: direct gradients), dh is kept for backward,
    which promises that only ``loss.sum()`` is differentiated."""

    @staticmethod
    def forward(ctx, h, fcw, fcb, labels, P, ncls, scale, gw, gb):
        N = h.shape[0]
        B, C = N // P, h.shape[-1]
        HW = h.numel() // (N * C)
        dev = h.device
        loss = torch.empty(P, dtype=torch.float32, device=dev)
        correct = torch.empty(P, dtype=torch.float32, device=dev)
        part = torch.empty(_lib.get_lib().mopt_resnet_head_part_floats(P, B, C),
                           dtype=torch.float32, device=dev)
        dh = torch.empty_like(h)
        _call("mopt_resnet_head", h.data_ptr(), fcw.data_ptr(), fcb.data_ptr(), labels.data_ptr(),
              P, B, HW, C, ncls, float(scale), 1, part.data_ptr(), dh.data_ptr(), gw.data_ptr(),
              gb.data_ptr(), loss.data_ptr(), correct.data_ptr(), _s(h))
        ctx.save_for_backward(dh)
        ctx.mark_non_differentiable(correct)
        ctx.set_materialize_grads(False)     # (no zero-filled gradient of `correct`)
        return loss, correct

    @staticmethod
    def backward(ctx, dloss, dcorrect):
        (dh,) = ctx.saved_tensors
        return dh, None, None, None, None, None, None, None, None


# the last block's BatchNorm 2 + shortcut + ReLU formed inside the classifier head
# (MOPT_BN_HEAD=0: the apply pass materialises the block output first)
_BN_HEAD = os.environ.get("MOPT_BN_HEAD", "1") != "0"


def bn_head_ok(pend: "PendingBN", fcw, fcb, labels) -> bool:
    """Whether ``bn_resnet_head`` has a kernel for this pending block output."""
    if not (_BN_HEAD and pend is not None and pend.sums is not None and pend.res is not None) \
            or pend.res_sub2 or pend.x.device.type != "cuda":
        return False
    x, P = pend.x, pend.P
    N, H, W, C = x.shape
    if tuple(pend.res.shape) != tuple(x.shape) or N % P or (N // P) % 16 or C % 8 or C > 64 or \
            16 % (C // 8) or tuple(fcw.shape) != (P, C, 16) or tuple(fcb.shape) != (P, 16) or \
            labels.dtype != torch.int64 or labels.numel() != N:
        return False
    nph = 16 // (C // 8)
    return (H * W) % (4 * nph) == 0 and (H * W) // (4 * nph) <= 8


class _BNHead(torch.autograd.Function):
    """The classifier head over relu(BN(x) + shortcut) of the last block, formed while pooling
    (csrc/resnet_head.hip ``head_kernel<true>``): the block output is never written.  The head
    writes dz -- the gradient behind the ReLU, which is also the block's shortcut gradient (to
    the mailbox) -- and the BatchNorm's reductions; backward is the BatchNorm's apply pass."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, running, fcw, fcb, labels, P, ncls, scale, gw, gb,
                sums, arena, bn_mailbox, eps, momentum):
        N, H, W, C = x.shape
        B, HW, M = N // P, H * W, x.numel() // (P * C)
        dev = x.device
        stat = torch.empty(P, 2, C, dtype=torch.float32, device=dev)
        fin = _BN_FIN_IN_CONV        # mean / rstd and the running update inside the head
        if not fin:
            _call("mopt_bn_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 0, 0,
                  stat.data_ptr(), running.data_ptr(), sums.data_ptr(), P, M, C, eps, momentum,
                  1, 1, 1, 0, 0, _s(x))
        loss = torch.empty(P, dtype=torch.float32, device=dev)
        correct = torch.empty(P, dtype=torch.float32, device=dev)
        part = torch.empty(_lib.get_lib().mopt_resnet_head_part_floats(P, B, C),
                           dtype=torch.float32, device=dev)
        dz = torch.empty_like(x)
        bwd_sums = arena.take(P * 2 * C).view(P, 2, C)
        _call("mopt_resnet_head_bn", x.data_ptr(), res.data_ptr(), stat.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), fcw.data_ptr(), fcb.data_ptr(),
              labels.data_ptr(), P, B, HW, C, ncls, float(scale), part.data_ptr(), dz.data_ptr(),
              gw.data_ptr(), gb.data_ptr(), loss.data_ptr(), correct.data_ptr(),
              bwd_sums.data_ptr(), sums.data_ptr() if fin else 0,
              running.data_ptr() if fin else 0, M, eps, momentum, _s(x))
        ctx.save_for_backward(x, dz, stat, gamma, beta)
        ctx.bwd_sums, ctx.P, ctx.bn_mailbox = bwd_sums, P, bn_mailbox
        ctx.grads = tuple(t.grad if (t.requires_grad and t.is_leaf and t.grad is not None) else None
                          for t in (gamma, beta))
        ctx.mark_non_differentiable(correct)
        ctx.set_materialize_grads(False)
        return loss, correct

    @staticmethod
    def backward(ctx, dloss, dcorrect):
        x, dz, stat, gamma, beta = ctx.saved_tensors
        P = ctx.P
        C = x.shape[-1]
        M = x.numel() // (P * C)
        dx = torch.empty_like(x)
        gg, gb = ctx.grads
        direct = gg is not None and gb is not None and gg.is_contiguous() and gb.is_contiguous()
        _call("mopt_bn_bwd", x.data_ptr(), 0, dz.data_ptr(), stat.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), dx.data_ptr(), 0, ctx.bwd_sums.data_ptr(),
              gg.data_ptr() if direct else 0, gb.data_ptr() if direct else 0, P, M, C, 0, 2,
              _s(x))
        if ctx.bn_mailbox is not None:
            ctx.bn_mailbox["dres"] = dz
            ctx.bn_mailbox["sub2"] = False
        dgamma = dbeta = None
        if not direct:
            dgamma = ctx.bwd_sums[:, 1].to(gamma.dtype)
            dbeta = ctx.bwd_sums[:, 0].to(gamma.dtype)
        return (dx, dgamma, dbeta) + (None,) * 15


def bn_resnet_head(pend: "PendingBN", fcw, fcb, labels, ncls, arena, scale=1.0, eps=1e-5,
                   momentum=0.1):
    """Training ``resnet_head(pend.materialize(arena), ...)`` with the pending block output
    formed inside the head (``_BNHead``); check ``bn_head_ok`` first."""
    if fcw.grad is None or fcb.grad is None:
        raise ValueError("bn_resnet_head writes into fcw.grad / fcb.grad")
    return _BNHead.apply(pend.x.contiguous(), pend.gamma.contiguous(), pend.beta.contiguous(),
                         pend.res.detach().contiguous(), pend.running, fcw, fcb,
                         labels.contiguous(), pend.P, ncls, scale, fcw.grad, fcb.grad, pend.sums,
                         arena, pend.mailbox, eps, momentum)


def resnet_head(h, fcw, fcb, labels, P, ncls, train, scale=1.0):
    """Per-trial loss sums and #correct of the classifier head over h [P*B, H, W, C] bf16 with
    fcw [P, C, NP], fcb [P, NP] (NP = 16 padded logits, the first ``ncls`` real) and labels
    [P*B] int64.  HIP: one fused kernel (+ a per-trial reduction); training writes dW / db
    straight into ``fcw.grad`` / ``fcb.grad`` (direct gradients) with ``scale`` applied."""
    if h.device.type != "cuda":
        loss, correct, _ = head_ref(h, fcw, fcb, labels, P, ncls)
        return loss, correct
    N, C = h.shape[0], h.shape[-1]
    if N % P or (N // P) % 16 or C % 8 or C > 64 or tuple(fcw.shape) != (P, C, 16) or \
            tuple(fcb.shape) != (P, 16) or labels.dtype != torch.int64 or labels.numel() != N:
        raise ValueError(f"resnet_head: h {tuple(h.shape)} fcw {tuple(fcw.shape)} fcb "
                         f"{tuple(fcb.shape)} labels {tuple(labels.shape)} {labels.dtype} P {P}")
    h = h.contiguous()
    labels = labels.contiguous()
    if train:
        if fcw.grad is None or fcb.grad is None:
            raise ValueError("resnet_head(train=True) writes into fcw.grad / fcb.grad")
        return _Head.apply(h, fcw, fcb, labels, P, ncls, scale, fcw.grad, fcb.grad)
    B, HW = N // P, h.numel() // (N * C)
    loss = torch.empty(P, dtype=torch.float32, device=h.device)
    correct = torch.empty(P, dtype=torch.float32, device=h.device)
    part = torch.empty(_lib.get_lib().mopt_resnet_head_part_floats(P, B, C),
                       dtype=torch.float32, device=h.device)
    _call("mopt_resnet_head", h.data_ptr(), fcw.data_ptr(), fcb.data_ptr(), labels.data_ptr(), P,
          B, HW, C, ncls, 1.0, 0, part.data_ptr(), None, None, None, loss.data_ptr(),
          correct.data_ptr(), _s(h))
    return loss, correct
