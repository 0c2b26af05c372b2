"""Host-side contracts of the population GEMM wrapper (ops/gemm.py): the f32 plan, the split-K
plan, and the CPU reference semantics of two-level batched operands and the epilogue
residual -- the same calls the K11 step makes (the GPU kernel is checked against them in
tests/test_pgemm_gpu.py)."""
import pytest
import torch

from metaopt_amd.ops.gemm import BIG_TILES, TILES, big_fits, f32_plan, pgemm, plan


@pytest.mark.parametrize("M,N,ta,want", [(1536, 768, False, 3), (1536, 4096, False, 4),
                                         (256, 768, True, 4), (384, 64, True, 3),
                                         (128, 32, False, 2), (128, 16, False, 1)])
def test_f32_plan_uses_64_row_tiles_without_split(M, N, ta, want):
    cfg, splits = f32_plan(M, N, ta)
    assert cfg == want and splits == 1
    assert cfg not in BIG_TILES


def test_plan_splits_short_grids_and_big_tiles_only_for_a_ragged_last_wave():
    cfg, splits, kps = plan(2, 64, 64, 8192)        # 2 output tiles: split the reduction
    assert splits > 1 and kps % 64 == 0 and splits * kps >= 8192
    cfg, splits, kps = plan(8, 4096, 4096, 1024)    # a big tile fills the chip: one K pass
    assert cfg in BIG_TILES and splits == 1 and kps == 1024
    # LM head dX: 384 long 256 x 256 tiles leave half the CUs idle in the second wave ->
    # 256 x 192 tiles (512 = 2 whole waves), or 2 K-splits when that tile is not available
    cfg, splits, kps = plan(8, 4096, 768, 32000)
    assert cfg == 11 and splits == 1
    from metaopt_amd.ops import gemm
    saved = gemm.BIG_TILES
    try:
        gemm.BIG_TILES = (5, 6, 7)
        assert plan(8, 4096, 768, 32000) == (5, 2, 16000)
    finally:
        gemm.BIG_TILES = saved
    # the other LM projections keep one K pass (the partials would cost more than the fill)
    for M, N, K in [(4096, 2304, 768), (768, 2304, 4096), (2048, 768, 4096), (768, 32000, 4096)]:
        assert plan(8, M, N, K)[1] == 1
    # an explicit K-split is honoured on the big tiles
    assert plan(8, 512, 512, 1024, 5, 4) == (5, 4, 256)
    for c in TILES:
        bm, bn = TILES[c]
        assert bm % 16 == 0 and bn % 16 == 0


def test_cpu_two_level_batch_with_broadcast_and_residual():
    torch.manual_seed(0)
    Po, I, M, N, K = 3, 2, 8, 16, 24
    x = torch.randn(Po, M, K)
    w = torch.randn(I, Po, K, N)
    out = torch.randn(Po, I, M, N)
    before = out.clone()
    a = x[:, None].expand(Po, I, M, K)               # inner dimension broadcast (stride 0)
    b = w.permute(1, 0, 2, 3)                        # strided inner dimension
    pgemm(a, b, out=out, res=out)
    ref = before + torch.einsum("pmk,ipkn->pimn", x, w)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_cpu_transposed_layouts_with_residual(ta, tb):
    torch.manual_seed(1)
    P, M, N, K = 2, 5, 8, 7
    A, B = torch.randn(P, M, K), torch.randn(P, K, N)
    a = A.transpose(1, 2).contiguous() if ta else A
    b = B.transpose(1, 2).contiguous() if tb else B
    r = torch.randn(P, M, N)
    out = pgemm(a, b, ta=ta, tb=tb, out=torch.empty(P, M, N), res=r)
    torch.testing.assert_close(out, torch.bmm(A, B) + r, rtol=1e-5, atol=1e-5)


def test_cpu_bn_into_conv_is_gpu_only():
    from metaopt_amd.ops import conv as cops
    x = torch.zeros(4, 8, 8, 16)
    w = torch.zeros(2, 9 * 16, 16)
    arena = object()
    assert not cops.bn_into_conv_ok(x, w, 2, 1, True, arena, True)


def test_measured_plans_override_the_model_for_their_shapes_only():
    """MEASURED_PLANS (profiles/r6/gemm/lm_tile_split_sweep.json) pick the measured-best tile of
    the LM's gate/up and attention-out weight gradients; other populations keep the model."""
    from metaopt_amd.ops.gemm import MEASURED_PLANS
    for (P, M, N, K), (cfg, sp) in MEASURED_PLANS.items():
        assert plan(P, M, N, K) == (cfg, sp, K // sp)
        assert big_fits(M, N, K, cfg)
    from metaopt_amd.ops.gemm import _plan_big
    assert plan(16, 768, 768, 4096) == _plan_big(16, 768, 768, 4096)    # not in the table
    assert plan(8, 768, 4096, 4096, cfg=6, splits=1) == (6, 1, 4096)   # explicit requests win
