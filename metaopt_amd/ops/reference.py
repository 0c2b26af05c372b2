"""Plain PyTorch references of the HIP kernels (CPU or GPU, fp32 math).

These define the semantics the gfx950 kernels must reproduce and serve three roles:
  * the numerics oracle of ``tests/test_kernels_gpu.py`` (kernel vs fp32 reference of the same op);
  * the CPU backend of :class:`metaopt_amd.ops.population.PopulationMLP` (BASELINE config 1, and
    every host-side test on machines without a GPU);
  * the "independent run" a batched population must reproduce trial by trial.

The dropout RNG is the counter-based murmur3-finaliser hash of ``csrc/common.h``; it is mirrored
here bit-for-bit with int64 arithmetic so masks are identical across backends.
"""
from __future__ import annotations

import math

import torch

M32 = 0xFFFFFFFF


def _mul32(h: torch.Tensor, c: int) -> torch.Tensor:
    """(h * c) mod 2**32 for int64 h in [0, 2**32) without int64 overflow."""
    lo = c & 0xFFFF
    hi = (c >> 16) & 0xFFFF
    return (h * lo + (((h * hi) & 0xFFFF) << 16)) & M32


def fmix32_t(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    h = h ^ (h >> 16)
    return h


def fmix32(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def rng_key(seed: int, layer: int, step: int) -> int:
    inner = (layer * 0x9E3779B9 + step * 0x7FEB352D + 0x632BE5AB) & M32
    return fmix32((seed & M32) ^ fmix32(inner))


def rng_uniform(key: int, idx: torch.Tensor) -> torch.Tensor:
    """U[0,1) float32 for int64 counters ``idx`` (same bits as ``rng_uniform`` in common.h)."""
    h = fmix32_t((_mul32(idx & M32, 0x9E3779B9)) ^ key)
    return (h >> 8).to(torch.float32) * (1.0 / 16777216.0)


def dropout_mask(seed: int, layer: int, step: int, rows: int, n: int, p: float,
                 device=None, row0: int = 0) -> torch.Tensor:
    """Keep-mask [rows, n] (bool) of the kernel's dropout for a padded output width ``n``."""
    r = torch.arange(row0, row0 + rows, device=device, dtype=torch.int64)
    c = torch.arange(n, device=device, dtype=torch.int64)
    idx = r[:, None] * n + c[None, :]
    u = rng_uniform(rng_key(seed, layer, step), idx)
    return u >= torch.tensor(p, dtype=torch.float32, device=device)


def bf16_weight(w: torch.Tensor) -> torch.Tensor:
    """The bf16 working copy the kernels read for an f32 master weight: the hi half of the
    split master (round to nearest, ties toward the smaller magnitude; csrc/common.h)."""
    return split_f32(w.float())[0].float()


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


def _inv_keep(drop: float) -> float:
    return float(torch.tensor(1.0, dtype=torch.float32) / (1.0 - torch.tensor(drop, dtype=torch.float32)))


def hidden_fwd(x, w, b, drop, seed, layer, step, emulate_bf16=True, train=True):
    """Reference of ``mlp_fwd_kernel``: dropout(relu(x w^T + b)), rounded to bf16 when emulating."""
    wq = bf16_weight(w) if emulate_bf16 else w
    z = torch.relu(x.float() @ wq.t() + b)
    if train and drop > 0.0:
        keep = dropout_mask(seed, layer, step, z.shape[0], z.shape[1], drop, device=z.device)
        z = torch.where(keep, z * _inv_keep(drop), torch.zeros_like(z))
    return bf16_round(z) if emulate_bf16 else z


def softmax_ce(logits: torch.Tensor, labels: torch.Tensor, n_real: int, inv_b: float,
               emulate_bf16: bool = True):
    """Reference of the fused CE epilogue: (loss_sum, correct, dlogits padded to logits' width)."""
    z = logits[:, :n_real].float()
    lse = torch.logsumexp(z, dim=1)
    loss = lse - z.gather(1, labels.long()[:, None])[:, 0]
    correct = (z.argmax(dim=1) == labels.long()).float()
    sm = torch.softmax(z, dim=1)
    onehot = torch.nn.functional.one_hot(labels.long(), n_real).float()
    g = torch.zeros_like(logits, dtype=torch.float32)
    g[:, :n_real] = (sm - onehot) * inv_b
    if emulate_bf16:
        g = bf16_round(g)
    return loss.sum(), correct.sum(), g


def split_f32(t: torch.Tensor):
    """f32 -> (hi bf16, lo int16): the split master of the HIP backend (csrc/common.h); hi is
    round-to-nearest with ties toward the smaller magnitude, (hi << 16) + lo - 0x7FFF the
    original bit pattern."""
    u = t.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    h = ((u + 0x7FFF) >> 16) & 0xFFFF
    lo = (u - (h << 16) + 0x7FFF) & 0xFFFF
    to16 = lambda x: (((x + 0x8000) & 0xFFFF) - 0x8000).to(torch.int16)  # noqa: E731
    return to16(h).view(torch.bfloat16), to16(lo)


def join_f32(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """(hi bf16, lo int16) -> the exact f32 master."""
    h = hi.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    l = lo.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    u = ((h << 16) + l - 0x7FFF) & 0xFFFFFFFF
    return (((u + 0x80000000) & 0xFFFFFFFF) - 0x80000000).to(torch.int32).view(torch.float32)


def sgd_update(w, m, g, lr, momentum, wd):
    """torch.optim.SGD(momentum, weight_decay, dampening=0, nesterov=False) on one tensor.
    A bf16 ``m`` is the kernel's bf16 momentum buffer: the f32 update is rounded once (RNE) and
    the rounded value drives the weight update."""
    g = g + wd * w
    if m.dtype == torch.bfloat16:
        m.copy_(m.float() * momentum + g)
        w.sub_(lr * m.float())
        return
    m.mul_(momentum).add_(g)
    w.sub_(lr * m)


def adamw_update(w, m, v, g, lr, b1, b2, eps, wd, t):
    """torch.optim.AdamW on one tensor (step ``t`` counted from 1)."""
    w.mul_(1.0 - lr * wd)
    m.mul_(b1).add_((1.0 - b1) * g)
    v.mul_(b2).add_((1.0 - b2) * g * g)
    bc1 = 1.0 - b1 ** t
    bc2 = 1.0 - b2 ** t
    denom = v.sqrt() / math.sqrt(bc2) + eps
    w.sub_((lr / bc1) * m / denom)


def init_layer(p32, m32, v32, w_off, b_off, K, N, k_real, n_real, seed, layer, bound):
    """Reference of ``mlp_init_kernel`` for one (member, layer): same RNG stream, same values."""
    dev = p32.device
    wkey = rng_key(seed, 0x1000 + layer, 0)
    bkey = rng_key(seed, 0x2000 + layer, 0)
    idx = torch.arange(N * K, device=dev, dtype=torch.int64)
    u = rng_uniform(wkey, idx)
    b32 = torch.tensor(bound, dtype=torch.float32, device=dev)
    w = (u * 2.0 - 1.0) * b32
    n = idx // K
    k = idx - n * K
    w = torch.where((n < n_real) & (k < k_real), w, torch.zeros_like(w))
    p32[w_off:w_off + N * K] = w
    bi = torch.arange(N, device=dev, dtype=torch.int64)
    bv = (rng_uniform(bkey, bi) * 2.0 - 1.0) * b32
    p32[b_off:b_off + N] = torch.where(bi < n_real, bv, torch.zeros_like(bv))
    m32[w_off:w_off + N * K] = 0
    m32[b_off:b_off + N] = 0
    if v32 is not None:
        v32[w_off:w_off + N * K] = 0
        v32[b_off:b_off + N] = 0
