"""The second-order-differentiable population GEMM (ops/pgemm_ad.py): every layout's value,
gradient, tangent and Hessian-vector product against plain torch.bmm (CPU, fp32 -- exact) and
against the fp32 reference on the GPU (bf16 MFMA kernel)."""
import pytest
import torch

from metaopt_amd.ops.pgemm_ad import matmul


def _f(mm, a, b, ta, tb):
    y = mm(a, b, ta, tb)
    return (torch.tanh(y) ** 2).sum()


def _bmm(a, b, ta, tb):
    return torch.bmm(a.transpose(1, 2) if ta else a, b.transpose(1, 2) if tb else b)


def _hvp(mm, a, b, ta, tb, va, vb):
    g = torch.func.grad(lambda a_, b_: _f(mm, a_, b_, ta, tb), argnums=(0, 1))
    (ga, gb), (ha, hb) = torch.func.jvp(g, (a, b), (va, vb))
    return ga, gb, ha, hb


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_forward_over_reverse_matches_bmm_cpu(ta, tb):
    torch.manual_seed(0)
    P, M, K, N = 2, 8, 16, 24
    a = torch.randn(P, *((K, M) if ta else (M, K)), dtype=torch.float64)
    b = torch.randn(P, *((N, K) if tb else (K, N)), dtype=torch.float64)
    va, vb = torch.randn_like(a), torch.randn_like(b)
    got = _hvp(matmul, a, b, ta, tb, va, vb)
    want = _hvp(_bmm, a, b, ta, tb, va, vb)
    for g, w in zip(got, want):
        torch.testing.assert_close(g, w, rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
def test_forward_over_reverse_on_the_mfma_kernel(ta, tb):
    torch.manual_seed(1)
    P, M, K, N = 3, 64, 128, 96
    dev = "cuda"
    a = torch.randn(P, *((K, M) if ta else (M, K)), device=dev) * 0.1
    b = torch.randn(P, *((N, K) if tb else (K, N)), device=dev) * 0.1
    va, vb = torch.randn_like(a) * 0.1, torch.randn_like(b) * 0.1
    got = _hvp(matmul, a, b, ta, tb, va, vb)
    want = _hvp(_bmm, a.double(), b.double(), ta, tb, va.double(), vb.double())
    for g, w in zip(got, want):
        err = (g.double() - w).abs().max().item()
        assert err <= 3e-2 * w.abs().max().item(), err
