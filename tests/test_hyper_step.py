"""The hand-derived stacked forward-over-reverse step (models/hyper_step.py) against torch.func:
the gradient and both Hessian-vector products of the op-by-op graph of ``lm_losses`` (jvp of
grad, vmapped over the tangents), and the plain (S = 1) gradient of the validation pass."""
import pytest
import torch

from metaopt_amd.models.hyper import HypergradLM, lm_losses
from metaopt_amd.models.hyper_step import SecondOrderStep, TorchStackOps
from metaopt_amd.models.llama import SyntheticLM


def _setup(P=2, B=2):
    torch.manual_seed(0)
    m = HypergradLM(P, "micro", batch_size=B, device="cpu", mode="func")
    m.reset(list(range(1, P + 1)), 0.3, 0.5)
    m.ze.normal_(0, 0.01)
    m.zm.normal_(0, 0.01)
    m.v.normal_(0, 0.01)
    data = SyntheticLM(512, 64, B, n_tokens=1 << 13, seed=0)
    tok, tgt = data.batch(0)
    return m, m._expand(tok), m._expand(tgt)


def _func_reference(m, tok, tgt):
    def loss_fn(W):
        per = lm_losses(m.params(W), tok, tgt, m.cfg, m.cos, m.sin)
        return per.sum(), per.detach()
    grad_fn = torch.func.grad_and_value(loss_fn, has_aux=True)

    def along(t):
        (g, (_, l)), (h, _) = torch.func.jvp(grad_fn, (m.w,), (t,))
        return g, l, h
    return torch.func.vmap(along, out_dims=(None, None, 0))(torch.stack([m.ze, m.zm]))


def _rel(a, b):
    return ((a - b).abs().max() / a.abs().max()).item()


def test_explicit_step_matches_torch_func_gradient_and_hvps():
    m, tok, tgt = _setup()
    g, losses, h = _func_reference(m, tok, tgt)
    st = SecondOrderStep(m.cfg, m.specs, m.offsets, m.P, 2, 3, "cpu", m.cos, m.sin)
    G = [torch.zeros_like(m.w) for _ in range(3)]
    l2 = st.run(m.w, [m.ze, m.zm], tok, tgt, G)
    torch.testing.assert_close(l2, losses, rtol=1e-6, atol=1e-6)
    assert _rel(g, G[0]) < 1e-5
    assert _rel(h[0], G[1]) < 1e-5
    assert _rel(h[1], G[2]) < 1e-5
    # every parameter tensor, not just the largest entries
    for (name, _, _), (o, k) in zip(m.specs, m.offsets):
        for a, b in ((g, G[0]), (h[0], G[1]), (h[1], G[2])):
            assert _rel(a[:, o:o + k], b[:, o:o + k]) < 1e-4, name


def test_plain_gradient_slice_equals_grad():
    m, tok, tgt = _setup()
    gref = torch.func.grad(lambda W: lm_losses(m.params(W), tok, tgt, m.cfg, m.cos,
                                               m.sin).sum())(m.w)
    st = SecondOrderStep(m.cfg, m.specs, m.offsets, m.P, 2, 1, "cpu", m.cos, m.sin)
    G = [torch.full_like(m.w, 7.0)]        # stale contents: every slice is (re)written
    st.run(m.w, [], tok, tgt, G)
    assert _rel(gref, G[0]) < 1e-5


def test_explicit_and_func_modes_train_identically():
    data = SyntheticLM(512, 64, 2, n_tokens=1 << 13, seed=0)
    out = {}
    for mode in ("explicit", "func"):
        m = HypergradLM(2, "micro", batch_size=2, device="cpu", mode=mode)
        m.reset([3, 4], 0.2, 0.7)
        for k in range(2):
            m.inner_step(*data.batch(k))
        out[mode] = (m.w.clone(), m.ze.clone(), m.zm.clone(), m.hypergradient(*data.validation()))
    for a, b in zip(out["explicit"][:3], out["func"][:3]):
        assert _rel(b, a) < 1e-4
    torch.testing.assert_close(out["explicit"][3][0], out["func"][3][0], rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(out["explicit"][3][1], out["func"][3][1], rtol=1e-5, atol=1e-6)


def test_shared_and_per_trial_token_batches():
    """tok/tgt expanded over the trials (stride 0) and materialised per trial give the same."""
    m, tok, tgt = _setup()
    st = SecondOrderStep(m.cfg, m.specs, m.offsets, m.P, 2, 3, "cpu", m.cos, m.sin)
    G1 = [torch.zeros_like(m.w) for _ in range(3)]
    G2 = [torch.zeros_like(m.w) for _ in range(3)]
    st.run(m.w, [m.ze, m.zm], tok, tgt, G1)
    st.run(m.w, [m.ze, m.zm], tok.contiguous(), tgt.contiguous(), G2)
    for a, b in zip(G1, G2):
        assert torch.equal(a, b)


def test_softmax_tangent_of_masked_rows():
    """The causal softmax tangent is zero on masked keys and sums to zero per row."""
    ops = TorchStackOps(3)
    N, T = 2, 8
    S1, S2 = torch.randn(N, 3 * T, T), torch.randn(N, T, 2 * T)
    Pm = torch.empty(N, 3 * T, T)
    ops.softmax_fwd(S1, S2, 0.5, Pm)
    mask = torch.ones(T, T, dtype=torch.bool).triu(1)
    for t in range(3):
        blk = Pm[:, t * T:(t + 1) * T]
        assert torch.all(blk[:, mask] == 0)
        target = torch.ones(N, T) if t == 0 else torch.zeros(N, T)
        torch.testing.assert_close(blk.sum(-1), target, atol=1e-6, rtol=0)


def test_layout_checks():
    m, tok, tgt = _setup()
    st = SecondOrderStep(m.cfg, m.specs, m.offsets, m.P, 2, 3, "cpu", m.cos, m.sin)
    with pytest.raises(ValueError, match="one layout"):
        st.run(m.w, [m.ze, m.zm.double()], tok, tgt, [torch.zeros_like(m.w)] * 3)
    with pytest.raises(ValueError, match="hip backend"):
        SecondOrderStep(m.cfg, m.specs, m.offsets, m.P, 2, 3, "cpu", m.cos, m.sin,
                        backend="hip")
