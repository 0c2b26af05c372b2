"""Population GEMM MFMA kernel (csrc/pgemm.hip) against fp32 PyTorch: every operand layout,
every tile configuration, ragged edges, split-K, and the autograd wrapper used by the LM/CNN."""
import pytest
import torch

from metaopt_amd.ops.gemm import LARGE_TILES, MF32_TILES, TILES, pbmm, pgemm, plan

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(P, M, N, K, ta, tb, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    A = torch.randn(P, M, K, device=DEV, generator=g).to(torch.bfloat16)
    B = torch.randn(P, K, N, device=DEV, generator=g).to(torch.bfloat16)
    a = A.transpose(1, 2).contiguous() if ta else A
    b = B.transpose(1, 2).contiguous() if tb else B
    return A, B, a, b


def _check(got, A, B):
    ref = torch.bmm(A.float(), B.float())
    err = (got.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale, (err, scale)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("P,M,N,K", [(3, 200, 136, 72), (2, 136, 16, 144), (2, 64, 40, 1000),
                                     (1, 8, 8, 8)])
def test_layouts_and_edges(ta, tb, P, M, N, K):
    A, B, a, b = _operands(P, M, N, K, ta, tb)
    _check(pgemm(a, b, ta=ta, tb=tb), A, B)


@pytest.mark.parametrize("cfg", sorted(c for c in TILES if c not in LARGE_TILES))
def test_every_tile_config(cfg):
    A, B, a, b = _operands(2, 264, 200, 136, False, True, seed=cfg)
    _check(pgemm(a, b, tb=True, cfg=cfg), A, B)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("cfg", [c for c in LARGE_TILES if c not in MF32_TILES])
def test_big_tiles_every_layout(cfg, ta, tb):
    """The 8-wave direct-to-LDS kernel (swizzled k-contiguous and row-contiguous images) in
    every operand layout; several K tiles so both LDS stages are used, distinct trials."""
    A, B, a, b = _operands(3, 512, 768, 384, ta, tb, seed=10 + cfg)   # N: 256, 192 and 128 | N
    assert plan(3, 512, 768, 384, cfg, 1)[0] == cfg
    _check(pgemm(a, b, ta=ta, tb=tb, cfg=cfg), A, B)


@pytest.mark.parametrize("cfg", MF32_TILES)
@pytest.mark.parametrize("P,M,N,K,splits", [(3, 512, 768, 384, 1), (300, 256, 768, 128, 1),
                                            (4, 256, 768, 2048, 4)])
def test_mfma32_tiles_nt(cfg, P, M, N, K, splits):
    """cfg 13 / 14 (pgemm_big32_kernel, v_mfma_f32_32x32x16_bf16, NT only): the 32 x 32 C layout
    through the permlane32 store and the split-K partial store; persistent walk over more tiles
    than workgroups (300 trials)."""
    A, B, a, b = _operands(P, M, N, K, False, True, seed=cfg + K)
    assert plan(P, M, N, K, cfg, splits)[:2] == (cfg, splits)
    _check(pgemm(a, b, tb=True, cfg=cfg, splits=splits), A, B)


def test_mfma32_tiles_refuse_other_layouts():
    A, B, a, b = _operands(2, 256, 256, 128, False, False, seed=1)
    with pytest.raises(RuntimeError):
        pgemm(a, b, cfg=13)
        torch.cuda.synchronize()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("P,M,N,K,splits", [(37, 512, 512, 256, 1), (5, 768, 1024, 1536, 1),
                                            (6, 512, 768, 2048, 2), (4, 256, 512, 1024, 4)])
def test_phased_tile(ta, tb, P, M, N, K, splits):
    """cfg 12 (pgemm_ph_kernel): 148 tiles on 148 workgroups, 120 tiles of 24 K-tiles, K-split
    partials over 4 and 2 splits -- and uneven tile counts per persistent workgroup (300 tiles:
    44 workgroups walk two)."""
    A, B, a, b = _operands(P, M, N, K, ta, tb, seed=P + K)
    assert plan(P, M, N, K, 12, splits)[:2] == (12, splits)
    _check(pgemm(a, b, ta=ta, tb=tb, cfg=12, splits=splits), A, B)
    if splits == 1 and P == 37:
        A, B, a, b = _operands(75, 512, 512, 128, ta, tb, seed=3)       # 300 tiles, 2 K-tiles
        _check(pgemm(a, b, ta=ta, tb=tb, cfg=12), A, B)


@pytest.mark.parametrize("cfg", [c for c in LARGE_TILES if c not in MF32_TILES])
def test_big_tiles_persistent_and_strided_output(cfg):
    """More tiles than workgroups (the persistent loop carries the next tile's first K-step
    across the epilogue), a C written into a wider row stride, split-K (f32 partials of the big
    tiles)."""
    A, B, a, b = _operands(2, 256, 256, 2048, True, False, seed=20 + cfg)
    _check(pgemm(a, b, ta=True, cfg=cfg, splits=4), A, B)
    wide = torch.zeros(2, 256, 384, dtype=torch.bfloat16, device=DEV)
    _check(pgemm(a, b, ta=True, cfg=cfg, out=wide[:, :, :256]), A, B)
    assert wide[:, :, 256:].abs().max().item() == 0     # nothing written past the view
    A, B, a, b = _operands(40, 512, 256, 128, False, True, seed=40 + cfg)   # 160-640 tiles
    _check(pgemm(a, b, tb=True, cfg=cfg), A, B)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("cfg,splits", [(5, 2), (5, 4), (6, 2), (7, 4)])
def test_big_tiles_split_k(cfg, splits, ta, tb):
    """K-split big tiles: every split starts its fills at its own K offset, writes f32 partials,
    the reduce pass sums them -- with more (tile, split) pairs than workgroups (persistent
    loop crossing split boundaries), into a wider output row stride."""
    A, B, a, b = _operands(24, 512, 512, 1024, ta, tb, seed=50 + cfg + splits)
    assert plan(24, 512, 512, 1024, cfg, splits)[:2] == (cfg, splits)
    wide = torch.zeros(24, 512, 640, dtype=torch.bfloat16, device=DEV)
    _check(pgemm(a, b, ta=ta, tb=tb, cfg=cfg, splits=splits, out=wide[:, :, :512]), A, B)
    assert wide[:, :, 512:].abs().max().item() == 0


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("splits", [1, 2])
def test_256x192_tile(ta, tb, splits):
    """The 256 x 192 big tile: 24-chunk row-contiguous images (lane-linear fills across k-rows,
    the 3-bit swizzle), 6 n-fragments per wave, persistent over 300 tiles, with and without a
    K-split."""
    A, B, a, b = _operands(25, 512, 1152, 256, ta, tb, seed=60 + splits)
    assert plan(25, 512, 1152, 256, 11, splits)[:2] == (11, splits)
    _check(pgemm(a, b, ta=ta, tb=tb, cfg=11, splits=splits), A, B)


def test_lm_head_dx_plan_splits_k():
    """The LM head's dX (K = 32000, 384 256 x 256 tiles on 256 CUs): the planner fills whole
    waves (256 x 192 tiles, or a K-split) and the split product matches."""
    cfg, splits, kps = plan(8, 4096, 768, 32000)
    assert cfg == 11 or splits == 2
    A, B, a, b = _operands(2, 512, 256, 32000, False, True, seed=77)
    _check(pgemm(a, b, tb=True, cfg=5, splits=2), A, B)


def test_big_tile_shape_guard():
    """A big tile on a shape it does not divide falls back (never launches out of bounds)."""
    A, B, a, b = _operands(1, 200, 256, 128, False, False, seed=30)
    _check(pgemm(a, b, cfg=5), A, B)


def test_split_k_reduction():
    P, M, N, K = 2, 256, 256, 4096
    assert plan(P, M, N, K)[1] > 1
    A, B, a, b = _operands(P, M, N, K, True, False, seed=3)
    _check(pgemm(a, b, ta=True), A, B)


def test_lm_shapes_exact_layouts():
    """The FFN down projection's input gradient (m 2048 x n 4096 x k 768 per trial, NT) -- the
    shape the library's transposed batched GEMM gets wrong -- and its weight gradient (TN)."""
    P, T, d, f = 2, 4096, 768, 2048
    A, B, a, b = _operands(P, T, f, d, False, True, seed=5)      # dX = dY[T, d] . W[f, d]^T
    _check(pgemm(a, b, tb=True), A, B)
    A, B, a, b = _operands(P, f, d, T, True, False, seed=6)      # dW = X^T[f, T] . dY[T, d]
    _check(pgemm(a, b, ta=True), A, B)


def test_pbmm_autograd_and_grad_out():
    torch.manual_seed(0)
    P, M, K, N = 3, 96, 64, 80
    x = torch.randn(P, M, K, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = torch.randn(P, K, N, device=DEV).to(torch.bfloat16).requires_grad_(True)
    buf = torch.zeros(P, K, N, dtype=torch.bfloat16, device=DEV)
    w.grad = buf
    y = pbmm(x, w, grad_out=w.grad)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    torch.bmm(xr, wr).backward(g.float())
    for got, ref in ((x.grad, xr.grad), (buf, wr.grad)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), err
    assert w.grad is buf           # written in place, never re-accumulated by autograd


@pytest.mark.parametrize("K,N", [(768, 2304), (768, 4096), (2048, 768), (768, 32000)])
def test_nn_forward_lm_shapes(K, N):
    """The LM's NN projection forwards (``nn_forward``) on the big-tile kernel."""
    from metaopt_amd.ops.gemm import nn_forward
    P, M = 2, 1024
    g = torch.Generator(device=DEV).manual_seed(K + N)
    x = (torch.randn(P, M, K, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    w = (torch.randn(P, K, N, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    _check(nn_forward(x, w), x, w)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("P,M,N,K,splits", [(3, 200, 136, 72, 1), (2, 64, 40, 1000, None)])
def test_f32_operands_and_output(ta, tb, P, M, N, K, splits):
    """f32 operands are rounded to bf16 while staged (bitwise the same products as casting
    first) and the f32 accumulators come back unrounded, also through split-K."""
    A, B, a, b = _operands(P, M, N, K, ta, tb, seed=7)
    a32, b32 = a.float(), b.float()
    got = pgemm(a32, b32, ta=ta, tb=tb, splits=splits)
    assert got.dtype == torch.float32
    _check(got, A, B)
    ref16 = pgemm(a, b, ta=ta, tb=tb, cfg=pgemm.__globals__["pick_tile"](M, N), splits=splits)
    # same inputs after rounding, same tile order: the bf16 path is the f32 result rounded
    assert torch.equal(got.to(torch.bfloat16), ref16)


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("splits", [None, 1, 2])
def test_f32_two_level_batch_broadcast_and_accumulate(ta, tb, splits):
    """4-D operands [Po, I, ., .] with a broadcast (stride-0) inner dim and strided slices, the
    f32 epilogue residual / in-place accumulation (res), with and without split-K -- the
    patterns of the K11 second-order step (models/hyper_step.py)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    Po, I, M, N, K = 3, 2, 72, 136, 256
    base_a = torch.randn(Po, 3, *((K, M) if ta else (M, K)), device=DEV, generator=g)
    a = base_a[:, :1].expand(-1, I, -1, -1)             # inner dim broadcast
    bb = torch.randn(I, Po, *((N, K) if tb else (K, N)), device=DEV, generator=g)
    b = bb.permute(1, 0, 2, 3)                           # inner stride = Po * K * N
    outbuf = torch.randn(Po, I + 1, M, N, device=DEV, generator=g)
    out = outbuf[:, 1:]                                  # strided output slices
    before, keep = out.clone(), outbuf[:, 0].clone()
    pgemm(a, b, ta=ta, tb=tb, out=out, res=out, splits=splits)
    assert torch.equal(outbuf[:, 0], keep)              # the slice outside out is untouched
    A = _bf(a.transpose(-1, -2) if ta else a)
    B = _bf(b.transpose(-1, -2) if tb else b)
    ref = before + torch.matmul(A, B)
    assert (out - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()
    # a separate residual (out = product + res), 3-D
    r = torch.randn(Po, M, N, device=DEV, generator=g)
    o3 = pgemm(base_a[:, 0], bb[0], ta=ta, tb=tb, out=torch.empty(Po, M, N, device=DEV),
               res=r, splits=splits)
    ref3 = r + torch.matmul(_bf(base_a[:, 0].transpose(-1, -2) if ta else base_a[:, 0]),
                            _bf(bb[0].transpose(-1, -2) if tb else bb[0]))
    assert (o3 - ref3).abs().max().item() <= 1e-3 * ref3.abs().max().item()


def test_res_requires_matching_layout():
    a = torch.randn(2, 64, 64, device=DEV)
    out = torch.empty(2, 64, 64, device=DEV)
    with pytest.raises(ValueError, match="res"):
        pgemm(a, a, out=out, res=torch.empty(2, 64, 64, device=DEV).transpose(1, 2))
