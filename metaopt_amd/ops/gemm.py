"""Population-batched GEMMs on the hand-written MFMA kernel (``csrc/pgemm.hip``).

``pgemm(a, b, ta, tb)`` computes ``C[p] = op(a[p]) @ op(b[p])`` for every trial ``p`` of the
population, reading each operand in the layout it is stored in (``ta``: ``a`` is stored
``[K, M]``; ``tb``: ``b`` is stored ``[N, K]``), so the backward GEMMs of a linear layer need no
transposed copies.  ``pbmm(x, w)`` is the differentiable ``x @ w`` of the LM and CNN paths:

* forward ``y = x w`` (NN), input gradient ``dx = dy w^T`` (NT), weight gradient
  ``dw = x^T dy`` (TN, split-K over the token / pixel dimension when the output tile grid is too
  small to fill the 256 CUs);
* ``grad_out``: the weight gradient is written straight into that buffer (the flat gradient
  buffer the fused optimizer reads) instead of being returned to autograd and accumulated.

The kernel replaced ``torch.bmm`` (hipBLASLt) in the backward, whose transposed-operand batched
bf16 GEMM returns wrong results for some shapes on the installed stack (``scripts/check_bmm.py``);
the copies that worked around it were ~20-40 % of the LM / ResNet step.  CPU tensors use ``torch.bmm`` (the
reference path of the tests).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional

import torch

from . import _lib

c_void_p, c_int, c_int64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64

_lib.register_signatures({
    "mopt_pgemm": ([c_void_p] * 4 + [c_int] * 7 + [c_int64] * 3 + [c_int] * 5 + [c_void_p],
                   c_int),
    "mopt_pgemm_f32": ([c_void_p] * 4 + [c_int] * 7 + [c_int64] * 3 + [c_int] * 5 + [c_void_p],
                       c_int),
    "mopt_pgemm_f32r": ([c_void_p] * 5 + [c_int] * 7 + [c_int64] * 3 + [c_int] * 5 + [c_void_p],
                        c_int),
    "mopt_pgemm_f32b": ([c_void_p] * 5 + [c_int] * 7 + [c_int64] * 3 + [c_int] * 6 +
                        [c_int64] * 3 + [c_void_p], c_int),
})

# tile configurations of csrc/pgemm.hip: cfg -> (BM, BN).  0-4: 4-wave register-staged kernel
# (any shape, ragged edges); 5-7: 8-wave direct-to-LDS kernel, one workgroup per CU, for shapes
# the tile divides (M % BM == N % BN == K % 64 == 0)
TILES = {0: (128, 128), 1: (128, 16), 2: (128, 32), 3: (64, 64), 4: (64, 128),
         5: (256, 256), 6: (256, 128), 7: (128, 256), 11: (256, 192), 12: (256, 256),
         13: (256, 256), 14: (256, 192)}
#: 256 x 192 (cfg 11): N = 768 outputs in 4 column panels, so the LM's N = 768 products fill
#: whole waves of 256 CUs (512 tiles for M = 4096, 256 for M = 2048) where 256 x 256 leaves a
#: 75 %-full last wave
BIG_TILES = (5, 6, 7, 11)
#: 12: the phased 256 x 256 kernel (pgemm_ph_kernel: fills in flight across the barriers, the two
#: wave rows staggered by a barrier); an even number of 64-deep K-tiles per split
PH_TILES = (12,)
#: 13 / 14: the big-tile kernel on the 32x32x16 MFMA (pgemm_big32_kernel), NT layout only (A
#: [M][K], B [N][K]); explicit requests only -- measured against 5 / 11 in profiles/round6.md
MF32_TILES = (13, 14)
LARGE_TILES = BIG_TILES + PH_TILES + MF32_TILES


def _ph_enabled() -> bool:
    return os.environ.get("MOPT_GEMM_PH", "0") != "0"

NUM_CU = 256
#: relative speed of the big tiles at equal occupancy of the chip; the 256 x 128 / 128 x 256 tiles
#: lose more on long reductions (less reuse per loaded byte): profiles/gemm_r2.md
BIG_SPEED = {5: 1.0, 6: 0.85, 7: 0.85, 11: 0.95, 12: 1.1}
LONG_K = 8192


def pick_tile(M: int, N: int) -> int:
    if N <= 16:
        return 1
    if N <= 32:
        return 2
    if N <= 64:
        return 3
    if M <= 64:
        return 4
    return 0


def f32_plan(M: int, N: int, ta: bool):
    """(tile cfg, splits) of an f32-operand GEMM (the K11 second-order step's shapes,
    profiles/r3/gemm32_k11.json): never split K -- the f32 partial tiles and the reduce pass
    cost more than the parallelism they add at these sizes (1.3-3.5x slower) -- and use the
    64-row tiles, whose 2-4x more workgroups fill the chip at P = 8..24 problems: 64 x 128 for
    weight gradients (TN) and wide outputs, 64 x 64 otherwise."""
    if N < 64:
        return pick_tile(M, N), 1
    if (ta and N >= 128) or N >= 2048:
        return 4, 1
    return 3, 1


def big_fits(M: int, N: int, K: int, cfg: int) -> bool:
    bm, bn = TILES[cfg]
    return M % bm == 0 and N % bn == 0 and K % (128 if cfg in PH_TILES else 64) == 0


#: model of the big kernel for the planner: sustained MFMA rate (FLOP/s at a full last wave) and
#: the HBM rate of the K-split partials (f32 written + read by the reduce pass, bf16 out)
BIG_RATE = 1.0e15
PART_BW = 4.0e12
MAX_BIG_SPLITS = 4
MIN_SPLIT_K = 1024


def _plan_big(P: int, M: int, N: int, K: int):
    """Best big tile and K-split by a time model: MFMA time at the tile's speed, scaled by the
    fraction of its last wave of 256 workgroups that is filled, plus the traffic of the f32
    partials when K is split (a split pays where few, long tiles leave CUs idle in the last
    wave, e.g. the LM head's dX: 384 tiles of K = 32000 on 256 CUs); None when no big tile
    divides the shape or fills the chip well."""
    best = None
    for cfg in BIG_TILES + (PH_TILES if _ph_enabled() else ()):
        if not big_fits(M, N, K, cfg):
            continue
        bm, bn = TILES[cfg]
        tiles = P * (M // bm) * (N // bn)
        speed = BIG_SPEED[cfg] * (0.8 if cfg in (6, 7) and K > LONG_K else 1.0)
        s = 1
        kq = 128 if cfg in PH_TILES else 64
        while s <= MAX_BIG_SPLITS:
            if K % (kq * s) or (s > 1 and K // s < MIN_SPLIT_K):
                break
            n = tiles * s
            fill = n / (math.ceil(n / NUM_CU) * NUM_CU)
            t = 2.0 * P * M * N * K / (BIG_RATE * speed * fill)
            if s > 1:
                t += P * M * N * (8.0 * s + 2.0) / PART_BW
            if best is None or t < best[0]:
                best = (t, cfg, s, fill)
            s *= 2
    if best is None or best[3] < 0.6:
        return None
    _, cfg, s, _ = best
    return cfg, s, K // s


#: measured exceptions to the planner's model, (P, M, N, K) -> (cfg, splits): the LM-125M
#: weight gradients whose best tile the fill model misjudges -- a persistent 1.5-wave tail runs
#: faster than its idle fraction suggests (profiles/r6/gemm/lm_tile_split_sweep.json, TFLOP/s):
#: gate/up dW 768 x 4096 x 4096 cfg 5 981 vs the modelled cfg 6 908; attention-out dW 768 x 768 x
#: 4096 cfg 7 650 vs cfg 11 split 2 590
MEASURED_PLANS = {(8, 768, 4096, 4096): (5, 1), (8, 768, 768, 4096): (7, 1)}


def plan(P: int, M: int, N: int, K: int, cfg: Optional[int] = None,
         splits: Optional[int] = None):
    """(tile cfg, splits, k_per_split) for a [P] x (M x K) . (K x N) problem: a big tile when it
    divides the shape and fills the chip, else a small one with the K reduction split when the
    output tiles alone give fewer than ~2 workgroups per CU."""
    if cfg is None and splits is None and (P, M, N, K) in MEASURED_PLANS:
        cfg, splits = MEASURED_PLANS[(P, M, N, K)]
        if big_fits(M, N, K, cfg) and K % (64 * splits) == 0:
            return cfg, splits, K // splits
        cfg = splits = None
    if cfg is None and splits is None:
        big = _plan_big(P, M, N, K)
        if big is not None:
            return big
    if cfg in LARGE_TILES:
        sp = splits or 1
        kq = 128 if cfg in PH_TILES else 64
        if big_fits(M, N, K, cfg) and K % (kq * sp) == 0:
            return cfg, sp, K // sp
        cfg = None                    # the tile does not divide this shape / this K-split
    cfg = pick_tile(M, N) if cfg is None else cfg
    bm, bn = TILES[cfg]
    blocks = P * math.ceil(M / bm) * math.ceil(N / bn)
    if splits is None:
        splits = 1
        if blocks < 2 * NUM_CU and K >= 512:
            splits = min(math.ceil(2 * NUM_CU / blocks), K // 256, 32)
    if splits <= 1:
        return cfg, 1, K
    kps = math.ceil(K / splits / 64) * 64
    return cfg, math.ceil(K / kps), kps


def _check_operand(t: torch.Tensor, name: str, dtype=torch.bfloat16) -> None:
    if t.dtype != dtype or t.dim() not in (3, 4) or t.stride(-1) != 1:
        raise ValueError(f"pgemm: {name} must be a [P, rows, cols] {dtype} tensor with unit "
                         f"column stride, got {t.dtype} {tuple(t.shape)} strides {t.stride()}")
    if t.shape[-1] % 8 or t.stride(-2) % 8 or \
            any(t.shape[i] > 1 and t.stride(i) % 8 for i in range(t.dim() - 2)) or \
            t.data_ptr() % 16:
        raise ValueError(f"pgemm: {name} rows must be 16-byte aligned multiples of 8 elements "
                         f"(shape {tuple(t.shape)}, strides {t.stride()})")


def pgemm(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False,
          out: Optional[torch.Tensor] = None, cfg: Optional[int] = None,
          splits: Optional[int] = None, res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out[p] = op(a[p]) @ op(b[p])`` in bf16 with f32 accumulation on the MFMA kernel.  f32
    operands give an f32 product: they are rounded to bf16 while the kernel stages them (no cast
    kernels) and the f32 accumulators are stored as they are.  ``res`` (f32 only, same shape and
    strides as ``out``, may be ``out`` itself): ``out = product + res`` in the epilogue -- a
    residual add or an in-place accumulation without a separate elementwise pass."""
    if a.device.type != "cuda":
        aa = a.transpose(-1, -2) if ta else a
        bb = b.transpose(-1, -2) if tb else b
        r = torch.matmul(aa.float(), bb.float())
        if res is not None:
            r = r + res
        r = r.to(out.dtype if out is not None else a.dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r
    f32 = a.dtype == torch.float32 or b.dtype == torch.float32
    dt = torch.float32 if f32 else torch.bfloat16
    if f32:
        a, b = a.float(), b.float()
    _check_operand(a, "a", dt)
    _check_operand(b, "b", dt)
    # 4-D operands [Po, I, rows, cols]: a two-level batch (any dim-0/1 strides, 0 = broadcast;
    # f32 only), flattened to P = Po * I problems
    four = a.dim() == 4
    if four != (b.dim() == 4) or (four and not f32):
        raise ValueError("pgemm: 4-D (two-level batch) operands must both be 4-D f32")
    lead = tuple(a.shape[:-2])
    K, M = (a.shape[-2], a.shape[-1]) if ta else (a.shape[-1], a.shape[-2])
    N, Kb = (b.shape[-2], b.shape[-1]) if tb else (b.shape[-1], b.shape[-2])
    if K != Kb or tuple(b.shape[:-2]) != lead:
        raise ValueError(f"pgemm: shape mismatch a {tuple(a.shape)} (ta={ta}) b "
                         f"{tuple(b.shape)} (tb={tb})")
    P = a.shape[0] * (a.shape[1] if four else 1)
    if N % 8:
        raise ValueError(f"pgemm: N = {N} must be a multiple of 8 (16-byte output rows)")
    if out is None:
        out = torch.empty(*lead, M, N, dtype=dt, device=a.device)
    elif tuple(out.shape) != (*lead, M, N) or out.stride(-1) != 1 or out.dtype != dt:
        raise ValueError(f"pgemm: out must be {(*lead, M, N)} {dt} row-major")
    _check_operand(out, "out", dt)
    if res is not None:
        if not f32 or res.dtype != torch.float32 or res.shape != out.shape or \
                res.stride() != out.stride():
            raise ValueError("pgemm: res must be an f32 tensor laid out exactly like out "
                             "(f32 operands only)")
    if f32 and cfg is None and splits is None:
        cfg, splits = f32_plan(M, N, ta)
    elif f32 and (cfg is None or cfg in LARGE_TILES):
        cfg = pick_tile(M, N)          # f32 operands: the register-staged tiles only
    cfg, splits, kps = plan(P, M, N, K, cfg, splits)
    part = (torch.empty(splits, P, M, N, dtype=torch.float32, device=a.device)
            if splits > 1 else None)
    pp = 0 if part is None else part.data_ptr()
    lib = _lib.get_lib()
    if four:
        _lib.check(lib.mopt_pgemm_f32b(
            a.data_ptr(), b.data_ptr(), out.data_ptr(), 0 if res is None else res.data_ptr(),
            pp, P, M, N, K, a.stride(2), b.stride(2), out.stride(2), a.stride(0), b.stride(0),
            out.stride(0), int(ta), int(tb), cfg, splits, kps, a.shape[1], a.stride(1),
            b.stride(1), out.stride(1), _lib.stream_ptr(a.device)), "pgemm")
        return out
    tail = (P, M, N, K, a.stride(1), b.stride(1), out.stride(1), a.stride(0), b.stride(0),
            out.stride(0), int(ta), int(tb), cfg, splits, kps, _lib.stream_ptr(a.device))
    if res is not None:
        _lib.check(lib.mopt_pgemm_f32r(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                       res.data_ptr(), pp, *tail), "pgemm")
    else:
        fn = lib.mopt_pgemm_f32 if f32 else lib.mopt_pgemm
        _lib.check(fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), pp, *tail), "pgemm")
    return out


def nn_forward(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Every product runs on pgemm: the big-tile kernel is at or above hipBLASLt on the LM's NN
    projections (profiles/gemm_r2.md, profiles/round3.md "LM GEMMs")."""
    return pgemm(a, b)


class _PBmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, grad_out):
        ctx.save_for_backward(a, b)
        ctx.grad_out = grad_out
        return nn_forward(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = pgemm(g, b, tb=True)
        if ctx.needs_input_grad[1]:
            if ctx.grad_out is not None:       # written in place: nothing to accumulate
                pgemm(a, g, ta=True, out=ctx.grad_out)
            else:
                db = pgemm(a, g, ta=True)
        return da, db, None


def pbmm(a: torch.Tensor, b: torch.Tensor, grad_out: Optional[torch.Tensor] = None):
    """Differentiable population GEMM ``a [P, M, K] @ b [P, K, N]``.  ``grad_out``: buffer that
    receives ``b``'s gradient directly (then autograd gets none for ``b``)."""
    if a.device.type != "cuda":
        return torch.bmm(a, b)
    return _PBmm.apply(a.contiguous(), b.contiguous(), grad_out)
