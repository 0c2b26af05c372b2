"""Numerics of the population-LM HIP kernels (attention, RMSNorm, RoPE, SwiGLU, cross-entropy,
embedding, fused AdamW) against fp32 PyTorch references of the same ops."""
import math

import numpy as np
import pytest
import torch

from metaopt_amd.ops import lm as ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("T,H,Bp", [(64, 1, 1), (256, 2, 3), (512, 4, 2)])
def test_attention_fwd_bwd(T, H, Bp):
    torch.manual_seed(0)
    q, k, v = (torch.randn(Bp, H, T, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
               for _ in range(3))
    do = torch.randn(Bp * T, H * 64, device=DEV).to(torch.bfloat16)
    o = ops.attention(q, k, v)
    o.backward(do)
    grads = [t.grad.clone() for t in (q, k, v)]
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ops.attention_ref(qr, kr, vr, 1 / 8)
    orf.backward(do.float())
    _close(o, orf, 2e-2)
    for g, r in zip(grads, (qr.grad, kr.grad, vr.grad)):
        _close(g, r, 3e-2)


def test_rmsnorm_fwd_bwd():
    torch.manual_seed(1)
    P, rpt, d = 3, 128, 768
    x = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(P, d, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    y = ops.rmsnorm(x, w, rpt)
    y.backward(dy)
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    yr = ops.rmsnorm_ref(xr, wr, rpt)
    yr.backward(dy.float())
    _close(y, yr, 1e-2)
    _close(x.grad, xr.grad, 2e-2)
    _close(w.grad, wr.grad, 2e-2)


@pytest.mark.parametrize("use_xs", [True, False])
def test_add_rmsnorm_fwd_bwd(use_xs):
    """Fused residual add + norm vs (x + delta, rmsnorm_ref) in fp32: outputs and the gradients
    of both summands and the weight, with and without a gradient flowing into the sum."""
    torch.manual_seed(4)
    P, rpt, d = 2, 128, 768
    x = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    dl = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(P, d, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    dxs = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    xs, y = ops.add_rmsnorm(x, dl, w, rpt)
    torch.autograd.backward([y, xs] if use_xs else [y], [dy, dxs] if use_xs else [dy])
    xr, dr, wr = (t.detach().float().requires_grad_(True) for t in (x, dl, w))
    xsr = xr + dr
    yr = ops.rmsnorm_ref(xsr, wr, rpt)
    torch.autograd.backward([yr, xsr] if use_xs else [yr],
                            [dy.float(), dxs.float()] if use_xs else [dy.float()])
    _close(xs, xsr, 1e-2)
    _close(y, yr, 1e-2)
    _close(x.grad, xr.grad, 2e-2)
    _close(dl.grad, dr.grad, 2e-2)
    _close(w.grad, wr.grad, 2e-2)


@pytest.mark.parametrize("use_xs", [True, False])
def test_rmsnorm_pass_joins_input_gradient(use_xs):
    """(x, rmsnorm(x)) with x also used downstream: the downstream gradient is added inside the
    norm's backward (dres) -- x.grad equals the fp32 sum of both paths."""
    torch.manual_seed(6)
    P, rpt, d = 2, 128, 768
    x = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(P, d, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    dxs = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    xo, y = ops.rmsnorm_pass(x, w, rpt)
    torch.autograd.backward([y, xo * 1] if use_xs else [y], [dy, dxs] if use_xs else [dy])
    xr, wr = (t.detach().float().requires_grad_(True) for t in (x, w))
    yr = ops.rmsnorm_ref(xr, wr, rpt)
    torch.autograd.backward([yr, xr * 1] if use_xs else [yr],
                            [dy.float(), dxs.float()] if use_xs else [dy.float()])
    assert torch.equal(xo, x)
    _close(y, yr, 1e-2)
    _close(x.grad, xr.grad, 2e-2)
    _close(w.grad, wr.grad, 2e-2)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("P,rpt,d", [(3, 1000, 768), (2, 48, 200)])
def test_rmsnorm_weight_grad_into_flat_view(fused, P, rpt, d):
    """Weight .grad preset to a bf16 view (the flat gradient buffer): the two-pass kernel
    (per-slice partials + reduce, no atomics) overwrites stale values with the gradient; row
    counts that do not divide into the slices and d not a multiple of the wave width."""
    torch.manual_seed(5)
    x = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    dl = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(P, d, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    w.grad = torch.full_like(w, 5.0)
    dy = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    wr = w.detach().float().requires_grad_(True)
    if fused:
        _, y = ops.add_rmsnorm(x, dl, w, rpt)
        yr = ops.rmsnorm_ref(x.float() + dl.float(), wr, rpt)
    else:
        y = ops.rmsnorm(x, w, rpt)
        yr = ops.rmsnorm_ref(x.float(), wr, rpt)
    y.backward(dy)
    yr.backward(dy.float())
    _close(w.grad, wr.grad, 2e-2)


def test_rope_split_roundtrip():
    torch.manual_seed(2)
    Bp, T, H = 2, 128, 3
    qkv = torch.randn(Bp * T, 3 * H * 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
    cos, sin = ops.rope_tables(T, device=DEV)
    q, k, v = ops.rope_split(qkv, cos, sin, T, H)
    qr, kr, vr = ops.rope_split_ref(qkv.detach(), cos, sin, T, H)
    for a, b in ((q, qr), (k, kr), (v, vr)):
        _close(a, b, 1e-2)
    g = [torch.randn_like(t) for t in (q, k, v)]
    torch.autograd.backward([q, k, v], g)
    xr = qkv.detach().float().requires_grad_(True)
    outs = ops.rope_split_ref(xr, cos, sin, T, H)
    torch.autograd.backward(list(outs), [t.float() for t in g])
    _close(qkv.grad, xr.grad, 2e-2)


def test_swiglu_fwd_bwd():
    torch.manual_seed(3)
    gu = torch.randn(2, 64, 2 * 704, device=DEV).to(torch.bfloat16).requires_grad_(True)
    dh = torch.randn(2, 64, 704, device=DEV).to(torch.bfloat16)
    h = ops.swiglu(gu)
    h.backward(dh)
    gr = gu.detach().float().requires_grad_(True)
    hr = ops.swiglu_ref(gr)
    hr.backward(dh.float())
    _close(h, hr, 1e-2)
    _close(gu.grad, gr.grad, 2e-2)


@pytest.mark.parametrize("V", [32000, 512, 4096 + 8])
def test_cross_entropy_loss_and_grad(V):
    torch.manual_seed(4)
    P, rpt = 2, 64
    logits = (3 * torch.randn(P * rpt, V, device=DEV)).to(torch.bfloat16)
    labels = torch.randint(0, V, (P * rpt,), device=DEV, dtype=torch.int32)
    lr_ = logits.float().requires_grad_(True)
    ref = ops.ce_ref(lr_, labels, rpt)
    (ref.sum() / rpt).backward()
    work = logits.clone().requires_grad_(True)
    loss = ops.cross_entropy(work, labels, rpt, grad_scale=1.0 / rpt)
    loss.sum().backward()
    _close(loss, ref, 1e-3)
    _close(work.grad, lr_.grad, 2e-2)
    ev = ops.ce_eval(logits.clone(), labels, rpt)
    _close(ev, ref, 1e-3)


def test_embedding_fwd_bwd():
    torch.manual_seed(5)
    P, V, d, rpt = 2, 1000, 256, 300
    table = torch.randn(P, V, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    tok = torch.randint(0, V, (P * rpt,), device=DEV, dtype=torch.int32)
    out = ops.embedding(tok, table, rpt)
    g = torch.randn_like(out)
    out.backward(g)
    tr = table.detach().float().requires_grad_(True)
    ref = ops.embed_ref(tok, tr, rpt)
    ref.backward(g.float())
    assert torch.equal(out, ref.to(torch.bfloat16))
    _close(table.grad, tr.grad, 1e-2)


@pytest.mark.parametrize("m_dtype", [torch.float32, torch.bfloat16])
def test_fused_adamw_matches_reference(m_dtype):
    """Fused AdamW vs the fp32 reference; with a bf16 first moment both round m once per
    update and use the unrounded value in the weight update."""
    torch.manual_seed(6)
    P = 3
    segments, off = [], 0
    for n in (768, 4096, 3000 * 8):
        segments.append((off, n))
        off += P * n
    bufs = {k: torch.randn(off, device=DEV) * (0.1 if k != "v" else 0.01) for k in ("p", "m", "v")}
    bufs["v"] = bufs["v"].abs()
    bufs["m"] = bufs["m"].to(m_dtype)
    g16 = torch.randn(off, device=DEV).to(torch.bfloat16)
    hp = np.zeros(P, dtype=ops.LM_HP_DTYPE)
    for p in range(P):
        hp[p] = (1e-3 * (p + 1), 0.9, 0.95, 1e-8, 0.1 * p, 1.0 if p != 1 else 0.0, 5 + p, 0)
    opt = ops.FlatAdamW(segments, P, DEV)
    hip = {k: v.clone() for k, v in bufs.items()}
    p16 = torch.empty(off, dtype=torch.bfloat16, device=DEV)
    opt.step(hip["p"], p16, g16, hip["m"], hip["v"], hp)
    ref = {k: v.clone().cpu() for k, v in bufs.items()}
    r16 = torch.empty(off, dtype=torch.bfloat16)
    ops.adamw_flat_ref(segments, P, ref["p"], r16, g16.cpu(), ref["m"], ref["v"], hp)
    torch.cuda.synchronize()
    for k in ("p", "m", "v"):
        # (a bf16 m may land one ulp apart where the f32 update sits on a rounding boundary)
        tol = dict(rtol=2 ** -7, atol=1e-6) if k == "m" and m_dtype == torch.bfloat16 else \
            dict(rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(hip[k].cpu(), ref[k], **tol)
    if m_dtype == torch.float32:
        assert torch.equal(p16.cpu(), r16)
    else:   # p32 agrees to f32 rounding; its bf16 copy may sit one ulp apart at a boundary
        torch.testing.assert_close(p16.cpu().float(), r16.float(), rtol=2 ** -7, atol=1e-6)
    assert hip["m"].dtype == m_dtype


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_fused_optimizer_split_master_matches_f32_master(kind):
    """The split master (p16 = high half, int16 low half; 22 B/param AdamW) updates exactly as
    the f32 master does: the joined result equals the f32 kernel's master bit for bit, and the
    working copy is the split's high half."""
    from metaopt_amd.ops.reference import join_f32, split_f32
    torch.manual_seed(8)
    P = 2
    segments, off = [], 0
    for n in (768, 4096 * 3):
        segments.append((off, n))
        off += P * n
    w = torch.randn(off, device=DEV) * 0.05
    m = (torch.randn(off, device=DEV) * 0.01).to(torch.bfloat16 if kind == "adamw"
                                                 else torch.float32)
    v = (torch.randn(off, device=DEV) * 0.01).abs() if kind == "adamw" else \
        torch.zeros(0, device=DEV)
    g16 = torch.randn(off, device=DEV).to(torch.bfloat16)
    hp = np.zeros(P, dtype=ops.LM_HP_DTYPE)
    for p in range(P):
        hp[p] = (1e-3 * (p + 1), 0.9, 0.95, 1e-8, 0.1 * p, 1.0 if p else 0.0, 3 + p, 0)
    opt = ops.FlatOptimizer(segments, P, DEV, kind=kind)
    ref = {"p": w.clone(), "m": m.clone(), "v": v.clone()}
    r16 = torch.empty(off, dtype=torch.bfloat16, device=DEV)
    opt.step(ref["p"], r16, g16, ref["m"], ref["v"], hp)
    hi, lo = split_f32(w)
    sm, sv = m.clone(), v.clone()
    opt.step(lo, hi, g16, sm, sv, hp)
    torch.cuda.synchronize()
    assert torch.equal(join_f32(hi, lo), ref["p"])
    assert torch.equal(hi, split_f32(ref["p"])[0])
    assert torch.equal(sm, ref["m"]) and torch.equal(sv, ref["v"])


def test_population_lm_step_matches_reference():
    from metaopt_amd.models.llama import PopulationLM, SyntheticLM
    from metaopt_amd.ops.population import MemberConfig
    data = SyntheticLM(512, 64, 4, n_tokens=1 << 14, seed=0, device=DEV)
    pops = []
    for dev in (DEV, "cpu"):
        pop = PopulationLM(2, "micro", batch_size=4, device=dev)
        for s in range(2):
            pop.set_member(s, MemberConfig(width=128, lr=2e-3 * (s + 1), momentum=0.9,
                                           seed=7 + s, beta2=0.95))
        pops.append(pop)
    # identical starting weights (the generators differ between devices)
    with torch.no_grad():
        pops[1].p32.copy_(pops[0].master_flat().cpu())
        pops[1].p16.copy_(pops[0].p16.cpu())
    losses = [[], []]
    for step in range(5):
        x, y = data.batch(step)
        for i, pop in enumerate(pops):
            pop.train_step(x.to(pop.device), y.to(pop.device))
            losses[i].append(pop.train_loss())
    a, b = np.array(losses[0]), np.array(losses[1])
    assert np.allclose(a, b, rtol=2e-2, atol=2e-2), (a, b)
    assert (a[-1] < a[0]).all()


def test_k11_hyper_kernels_match_reference():
    from metaopt_amd.models.hyper import HypergradLM, hyper_sgdm_ref
    torch.manual_seed(8)
    P, n = 3, 4096 + 64
    bufs = [torch.randn(P, n, device=DEV) for _ in range(9)]
    eta = torch.tensor([0.1, 0.05, 0.3], device=DEV)
    mu = torch.tensor([0.9, 0.5, 0.0], device=DEV)
    ref = [b.clone() for b in bufs]
    hyper_sgdm_ref(*ref, eta, mu)
    m = HypergradLM.__new__(HypergradLM)
    m.device, m.P, m.n = torch.device(DEV), P, n
    m.w, m.v, m.ze, m.zm, m.ye, m.ym = bufs[:6]
    m.eta, m.mu = eta, mu
    m._update(*bufs[6:])
    torch.cuda.synchronize()
    for a, b in zip(bufs[:6], ref[:6]):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)


def test_hypergradient_on_gpu_matches_cpu():
    from metaopt_amd.models.hyper import HypergradLM
    from metaopt_amd.models.llama import SyntheticLM
    out = []
    for dev in (DEV, "cpu"):
        data = SyntheticLM(512, 64, 2, n_tokens=1 << 13, seed=0, device=dev)
        m = HypergradLM(2, "micro", batch_size=2, device=dev)
        m.reset([1, 2], 0.3, 0.5)
        if dev == "cpu":
            m.w.copy_(out[0][2])
        w0 = m.w.detach().clone().cpu()
        for k in range(3):
            m.inner_step(*data.batch(k))
        hg, vl = m.hypergradient(*data.validation())
        out.append((hg.cpu(), vl.cpu(), w0))
    torch.testing.assert_close(out[0][0], out[1][0], rtol=5e-2, atol=5e-3)
    torch.testing.assert_close(out[0][1], out[1][1], rtol=1e-3, atol=1e-3)


def test_fused_adamw_at_125m_layout_is_finite_and_exact_on_samples():
    """The 125M-LM segment layout (8 trials, ~1.07B elements): no NaN, and every segment's first
    trial and last trial match the reference."""
    from metaopt_amd.models.llama import PRESETS, param_specs
    P = 8
    segments, off = [], 0
    for _, shape, _ in param_specs(PRESETS["llama-125m"]):
        n = int(np.prod(shape))
        segments.append((off, n))
        off += P * n
    g = torch.Generator(device=DEV).manual_seed(0)
    p32 = torch.randn(off, device=DEV, generator=g) * 0.02
    g16 = (torch.randn(off, device=DEV, generator=g) * 1e-3).to(torch.bfloat16)
    m = torch.zeros(off, device=DEV)
    v = torch.zeros(off, device=DEV)
    p16 = torch.empty(off, dtype=torch.bfloat16, device=DEV)
    hp = np.zeros(P, dtype=ops.LM_HP_DTYPE)
    for p in range(P):
        hp[p] = (3e-4 * (p + 1), 0.9, 0.95, 1e-8, 0.1, 1.0, 1, 0)
    before = p32.clone()
    ops.FlatOptimizer(segments, P, DEV).step(p32, p16, g16, m, v, hp)
    torch.cuda.synchronize()
    assert torch.isfinite(p32).all() and torch.isfinite(m).all() and torch.isfinite(v).all()
    # reference on a subset: all segments, trials 0 and P-1 (clipping uses the full trial norm)
    sumsq = torch.zeros(P, dtype=torch.float64, device=DEV)
    for o, n in segments:
        sumsq += g16[o:o + P * n].view(P, n).double().pow(2).sum(1)
    for o, n in segments:
        for p in (0, P - 1):
            sl = slice(o + p * n, o + (p + 1) * n)
            nrm = float(sumsq[p].sqrt())
            scale = 1.0 / (nrm + 1e-6) if nrm > 1.0 else 1.0
            gr = g16[sl].float() * scale
            lr, b1, b2, eps, wd = (float(hp[p][k]) for k in ("lr", "b1", "b2", "eps", "wd"))
            mm = (1 - b1) * gr
            vv = (1 - b2) * gr * gr
            w = before[sl] * (1 - lr * wd) - lr / (1 - b1) * mm / (vv.sqrt() / (1 - b2) ** 0.5 + eps)
            torch.testing.assert_close(p32[sl], w, rtol=1e-4, atol=1e-6)


def test_embedding_backward_into_flat_gradient_sorted():
    """With the table's .grad preset (the flat gradient buffer), the backward sorts the
    (trial, token) keys and writes every touched row once: equal to the fp32 reference
    (heavily repeated tokens included), untouched rows zero, deterministic across runs."""
    torch.manual_seed(8)
    P, V, d, rpt = 3, 512, 768, 1024
    table = torch.randn(P, V, d, device=DEV).to(torch.bfloat16).requires_grad_(True)
    table.grad = torch.full_like(table, 7.0)               # stale values must be overwritten
    tok = torch.randint(0, 64, (P * rpt,), device=DEV, dtype=torch.int32)   # many repeats
    g = torch.randn(P * rpt, d, device=DEV).to(torch.bfloat16)
    grads = []
    for _ in range(2):
        out = ops.embedding(tok, table, rpt)
        out.backward(g)
        grads.append(table.grad.clone())
    assert torch.equal(grads[0], grads[1])
    tr = table.detach().float().requires_grad_(True)
    ops.embed_ref(tok, tr, rpt).backward(g.float())
    _close(grads[0], tr.grad, 1e-2)
    assert (grads[0][:, 64:] == 0).all()


@pytest.mark.parametrize("P,R,d,F,big", [(8, 2048, 256, 512, True), (2, 64, 64, 64, False)])
def test_swiglu_mlp_epilogues_match_reference(P, R, d, F, big):
    """swiglu(h @ wgu) @ wdown with the SwiGLU in the gate/up GEMM's epilogue (gate / up
    interleaved in 16-column groups; pgemm.hip EPI 1) -- or, on shapes without a big tile, the
    GEMM + interleaved swiglu kernel -- against fp32 autograd: output and the gradients of h,
    wgu and wdown (backward: GEMMs + the interleaved swiglu backward kernel)."""
    from metaopt_amd.ops.gemm import LARGE_TILES, plan
    torch.manual_seed(3)
    assert (plan(P, R, 2 * F, d)[0] in LARGE_TILES) == big
    h = (torch.randn(P, R, d, device=DEV) * 0.5).to(torch.bfloat16)
    wgu = (torch.randn(P, d, 2 * F, device=DEV) / d ** 0.5).to(torch.bfloat16)
    wdown = (torch.randn(P, F, d, device=DEV) / F ** 0.5).to(torch.bfloat16)
    dy = torch.randn(P, R, d, device=DEV).to(torch.bfloat16)
    hs, gs, ds = (t.clone().requires_grad_(True) for t in (h, wgu, wdown))
    y = ops.swiglu_mlp(hs, gs, ds)
    y.backward(dy)
    hr, gr, dr = (t.float().clone().requires_grad_(True) for t in (h, wgu, wdown))
    yr = torch.bmm(ops.swiglu_ref(torch.bmm(hr, gr), il=True), dr)
    yr.backward(dy.float())
    torch.cuda.synchronize()

    def rel(a, b):
        return float((a.float() - b).norm() / b.norm())
    assert rel(y, yr) < 2e-2, rel(y, yr)
    for got, ref in ((hs.grad, hr.grad), (gs.grad, gr.grad), (ds.grad, dr.grad)):
        assert rel(got, ref) < 3e-2, rel(got, ref)


@pytest.mark.parametrize("P,B,T,H,big", [(8, 4, 512, 4, True), (2, 2, 64, 2, False)])
def test_qkv_rope_epilogue_matches_reference(P, B, T, H, big):
    """q, k, v = rope(h @ wqkv) with interleaved RoPE pairs applied in the QKV GEMM's epilogue
    (pgemm.hip EPI 3) -- or, without a big tile, the GEMM + the interleaved RoPE kernel --
    against fp32 autograd of rope_split_ref(il=True): the three head tensors and the gradients
    of h and wqkv."""
    from metaopt_amd.ops.gemm import LARGE_TILES, plan
    torch.manual_seed(9)
    d, R = 64 * H, B * T
    assert (plan(P, R, 3 * d, d)[0] in LARGE_TILES) == big
    h = (torch.randn(P, R, d, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(P, d, 3 * d, device=DEV) / d ** 0.5).to(torch.bfloat16)
    cos, sin = ops.rope_tables(T, device=DEV)
    hs, ws = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    outs = ops.qkv_rope(hs, ws, cos, sin, T, H)
    gs = [torch.randn_like(o) for o in outs]
    torch.autograd.backward(list(outs), gs)
    hr, wr = h.float().requires_grad_(True), w.float().requires_grad_(True)
    refs = ops.rope_split_ref(torch.bmm(hr, wr).reshape(P * R, 3 * d), cos, sin, T, H, il=True)
    torch.autograd.backward(list(refs), [g.float() for g in gs])
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert o.shape == r.shape
        _close(o, r, 2e-2)
    _close(hs.grad, hr.grad, 3e-2)
    _close(ws.grad, wr.grad, 3e-2)


def test_qkv_rope_attention_matches_reference():
    """The fused node (QKV GEMM with the RoPE epilogue, attention, and the attention backward
    writing the QKV gradient with the inverse RoPE) against fp32 autograd of the unfused
    reference: output and the gradients of h and wqkv."""
    torch.manual_seed(10)
    P, B, T, H = 4, 2, 256, 2
    d, R = 64 * H, B * T
    h = (torch.randn(P, R, d, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(P, d, 3 * d, device=DEV) / d ** 0.5).to(torch.bfloat16)
    cos, sin = ops.rope_tables(T, device=DEV)
    hs, ws = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    o = ops.qkv_rope_attention(hs, ws, cos, sin, T, H)
    g = torch.randn_like(o)
    o.backward(g)
    hr, wr = h.float().requires_grad_(True), w.float().requires_grad_(True)
    q, k, v = ops.rope_split_ref(torch.bmm(hr, wr).reshape(P * R, 3 * d), cos, sin, T, H, il=True)
    orf = ops.attention_ref(q, k, v, 0.125)
    orf.backward(g.float())
    torch.cuda.synchronize()
    _close(o, orf, 2e-2)
    _close(hs.grad, hr.grad, 3e-2)
    _close(ws.grad, wr.grad, 3e-2)
