"""Forward-mode hypergradients through SGD-momentum (config 4): exactness against finite
differences, the outer sweep, and the C2 all-reduce across gloo ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from metaopt_amd.models.hyper import HypergradientSweep, HypergradLM, hyper_sgdm_ref
from metaopt_amd.models.llama import SyntheticLM


def _data(batch=2):
    return SyntheticLM(512, 64, batch, n_tokens=1 << 13, seed=0)


def _val_after(m, data, lr, mu, K=3):
    m.reset([1, 2], lr, mu)
    for k in range(K):
        m.inner_step(*data.batch(k))
    return m.hypergradient(*data.validation())


def test_hypergradient_matches_finite_differences():
    torch.manual_seed(0)
    m = HypergradLM(2, "micro", batch_size=2, device="cpu")
    data = _data()
    hg, _ = _val_after(m, data, 0.4, 0.6)
    eps = 1e-3
    _, vp = _val_after(m, data, 0.4 + eps, 0.6)
    _, vm = _val_after(m, data, 0.4 - eps, 0.6)
    torch.testing.assert_close(hg[:, 0], (vp - vm) / (2 * eps), rtol=2e-2, atol=2e-3)
    _, vp = _val_after(m, data, 0.4, 0.6 + eps)
    _, vm = _val_after(m, data, 0.4, 0.6 - eps)
    torch.testing.assert_close(hg[:, 1], (vp - vm) / (2 * eps), rtol=2e-2, atol=2e-3)


def test_k11_reference_update_semantics():
    P, n = 2, 8
    z = lambda: torch.zeros(P, n)  # noqa: E731
    w, v, ze, zm, ye, ym = torch.ones(P, n), z(), z(), z(), z(), z()
    g = torch.full((P, n), 2.0)
    eta, mu = torch.tensor([0.1, 0.2]), torch.tensor([0.5, 0.9])
    hyper_sgdm_ref(w, v, ze, zm, ye, ym, g, z(), z(), eta, mu)
    assert torch.allclose(v, g)
    assert torch.allclose(w[:, 0], 1 - eta * 2)
    assert torch.allclose(ze[:, 0], torch.full((P,), -2.0))   # d w / d eta = -v'
    assert torch.allclose(zm, z())                              # v was 0


def test_outer_sweep_records_trials():
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    exp = build_experiment("hyper", priors={"/lr": "loguniform(1e-3, 1)",
                                            "/momentum": "uniform(0, 0.99)"},
                           storage=DocumentStorage(EphemeralDB()))
    m = HypergradLM(2, "micro", batch_size=2, device="cpu")
    sweep = HypergradientSweep(m, _data(), experiment=exp, lr0=0.05, mu0=0.5, meta_lr=0.2,
                               inner_steps=3)
    hist = sweep.run(3)
    assert len(hist) == 3 and all(h["val_loss"] > 0 for h in hist)
    assert hist[1]["lr"] != hist[0]["lr"]
    trials = exp.fetch_trials()
    assert len(trials) == 3
    assert all(t.objective is not None and t.gradient is not None for t in trials)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _c2_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from metaopt_amd.parallel.comm import init_from_env
    comm = init_from_env(backend="gloo")
    m = HypergradLM(1, "micro", batch_size=2, device="cpu")
    sweep = HypergradientSweep(m, _data(), comm=comm, lr0=0.05, mu0=0.5, meta_lr=0.2,
                               inner_steps=2)
    hist = sweep.run(2)
    q.put((rank, [h["lr"] for h in hist], [h["d_lr"] for h in hist], list(sweep.theta)))
    dist.destroy_process_group()


def test_c2_allreduce_keeps_ranks_in_lockstep_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    (_, lr0, g0, th0), (_, lr1, g1, th1) = res
    assert lr0 == lr1 and g0 == g1 and th0 == th1   # identical meta-steps on every rank


def _dp_worker(rank, world, port, q):
    """C3: 2 ranks, each with half of every minibatch, data-parallel over the same runs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from metaopt_amd.parallel.comm import init_from_env
    comm = init_from_env(backend="gloo")
    data = _data(batch=4)
    m = HypergradLM(2, "micro", batch_size=2, device="cpu", dp_comm=comm)
    m.reset([1, 2], 0.3, 0.6)
    for k in range(3):
        tok, tgt = data.batch(k)
        m.inner_step(tok[2 * rank:2 * rank + 2], tgt[2 * rank:2 * rank + 2])
    vt, vg = data.validation()
    hg, vl = m.hypergradient(vt, vg)
    q.put((rank, m.w.numpy().copy(), hg.numpy().copy(), vl.numpy().copy()))  # by value
    dist.destroy_process_group()


def test_c3_intra_trial_data_parallel_equals_one_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    torch.set_num_threads(2)
    data = _data(batch=4)
    m = HypergradLM(2, "micro", batch_size=4, device="cpu")
    m.reset([1, 2], 0.3, 0.6)
    for k in range(3):
        m.inner_step(*data.batch(k))
    hg, vl = m.hypergradient(*data.validation())
    (_, w0, hg0, vl0), (_, w1, hg1, vl1) = [(r, *map(torch.from_numpy, t)) for r, *t in res]
    assert torch.equal(w0, w1) and torch.equal(hg0, hg1)     # the DP ranks stay identical
    torch.testing.assert_close(w0, m.w, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(hg0, hg, rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(vl0, vl, rtol=1e-5, atol=1e-6)


def test_analytic_functions_match_op_by_op_second_order():
    """The K11 graph's hand-derived Functions (parameter unflatten, RoPE, causal softmax) give
    the same values, gradients and Hessian-vector products (jvp of grad, vmapped over two
    tangents) as the op-by-op expressions they replace."""
    import math
    from metaopt_amd.models.hyper import _CausalSoftmax, rope_split
    from metaopt_amd.ops import lm as lmops
    torch.manual_seed(0)
    T, H, Bp = 16, 2, 3
    qkv = torch.randn(Bp * T, 3 * H * 64, dtype=torch.float32)
    cos, sin = lmops.rope_tables(T)
    scale = 1.0 / math.sqrt(64)

    def attn(q, k, v, soft):
        s = q @ k.transpose(-1, -2)
        return soft(s) @ v

    def soft_ref(s):
        mask = torch.ones(T, T, dtype=torch.bool).triu(1)
        return (s * scale).masked_fill(mask, float("-inf")).softmax(-1)

    def f_new(z):
        q, k, v = rope_split(z, cos, sin, T, H)
        return (attn(q, k, v, lambda s: _CausalSoftmax.apply(s, scale)) ** 2).sum()

    def f_ref(z):
        q, k, v = lmops.rope_split_ref(z, cos, sin, T, H)
        return (attn(q, k, v, soft_ref) ** 2).sum()

    assert torch.allclose(f_new(qkv), f_ref(qkv), rtol=1e-5)
    tangents = torch.randn(2, *qkv.shape, dtype=torch.float32)

    def hvp(f):
        along = lambda t: torch.func.jvp(torch.func.grad(f), (qkv,), (t,))
        return torch.func.vmap(along)(tangents)

    (g1, h1), (g2, h2) = hvp(f_new), hvp(f_ref)
    assert torch.allclose(g1, g2, rtol=1e-4, atol=1e-4)
    assert torch.allclose(h1, h2, rtol=1e-4, atol=1e-4)


def test_swiglu_and_rmsnorm_match_reference_second_order():
    from metaopt_amd.models.hyper import _SwiGLU, rmsnorm
    from metaopt_amd.ops import lm as lmops
    torch.manual_seed(1)
    P, rpt, d = 2, 8, 32
    gu = torch.randn(P, rpt, 2 * d)
    x = torch.randn(P * rpt, d)
    w = 1 + 0.1 * torch.randn(P, d)
    assert torch.equal(rmsnorm(x, w, rpt, 1e-5), lmops.rmsnorm_ref(x, w, rpt, 1e-5))
    f_new = lambda z: (_SwiGLU.apply(z) ** 2).sum()
    f_ref = lambda z: (lmops.swiglu_ref(z) ** 2).sum()
    assert torch.allclose(f_new(gu), f_ref(gu), rtol=1e-6)
    tangents = torch.randn(2, *gu.shape)
    hvp = lambda f: torch.func.vmap(
        lambda t: torch.func.jvp(torch.func.grad(f), (gu,), (t,)))(tangents)
    (g1, h1), (g2, h2) = hvp(f_new), hvp(f_ref)
    assert torch.allclose(g1, g2, rtol=1e-5, atol=1e-5)
    assert torch.allclose(h1, h2, rtol=1e-5, atol=1e-5)


def _fd_population(dev, eta=0.3, mu=0.5, h=1e-3, steps=3, w0=None):
    """Five inner runs from ONE initialisation on the same batches: (eta, mu) and its central
    finite-difference neighbours in eta and in mu.  Returns the hypergradient of run 0, the
    finite differences and the initial weights (``w0``: start from these instead -- the CPU
    and GPU generators draw different initialisations from one seed)."""
    from metaopt_amd.models.hyper import HypergradLM
    from metaopt_amd.models.llama import SyntheticLM
    data = SyntheticLM(512, 64, 2, n_tokens=1 << 13, seed=0, device=dev)
    m = HypergradLM(5, "micro", batch_size=2, device=dev)
    m.reset([7] * 5, [eta, eta + h, eta - h, eta, eta], [mu, mu, mu, mu + h, mu - h])
    if w0 is not None:
        m.w.copy_(w0.to(m.w.device))
    w_init = m.w.detach().clone().cpu()
    for k in range(steps):
        m.inner_step(*data.batch(k))
    hg, vl = m.hypergradient(*data.validation())
    vl = vl.double().cpu()
    fd = torch.tensor([(vl[1] - vl[2]) / (2 * h), (vl[3] - vl[4]) / (2 * h)])
    return hg[0].double().cpu(), fd, w_init


def test_hypergradient_matches_central_finite_difference_fp32():
    """d L_val / d(lr, momentum) of the forward-mode unrolled hypergradient equals the central
    finite difference of the fp32 validation loss after the same 3 inner steps (CPU, fp32
    throughout: the check of the derivation itself)."""
    hg, fd, _ = _fd_population("cpu")
    assert fd.abs().max() > 1e-2                      # a non-trivial derivative
    torch.testing.assert_close(hg, fd, rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_gpu_hypergradient_matches_fp32_finite_difference():
    """The HIP path (bf16-operand MFMA GEMMs, f32 accumulation, f32 activations / state) against
    the central finite difference of the fp32 CPU validation loss: the tolerance is the bf16
    operand rounding of the GEMMs (5 % relative)."""
    hg, _, w0 = _fd_population("cuda")
    _, fd, _ = _fd_population("cpu", w0=w0)
    torch.testing.assert_close(hg, fd, rtol=5e-2, atol=5e-3)
