"""Layer-by-layer comparison of the population LM forward on the HIP ops vs the fp32 references."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.models.llama import PopulationLM, SyntheticLM  # noqa: E402
from metaopt_amd.ops import lm as ops  # noqa: E402
from metaopt_amd.ops.population import MemberConfig  # noqa: E402

pop = PopulationLM(2, "micro", batch_size=4, device="cuda")
for s in range(2):
    pop.set_member(s, MemberConfig(width=128, lr=1e-3, seed=7 + s, beta2=0.95))
data = SyntheticLM(512, 64, 4, n_tokens=1 << 14, seed=0, device="cuda")
x, y = data.batch(0)
tok, tgt = pop._expand(x), pop._expand(y)
c, P, W = pop.cfg, pop.capacity, pop.W
T, d, H = c.seq_len, c.d_model, c.n_heads
rpt = tok.numel() // P
R = tok.numel()


def rep(name, a, b):
    a, b = a.float(), b.float()
    print(f"{name:12s} nan={torch.isnan(a).any().item()} inf={torch.isinf(a).any().item()} "
          f"maxerr={(a - b).abs().max().item():.4g} scale={b.abs().max().item():.4g}", flush=True)


with torch.no_grad():
    print("p16 finite:", torch.isfinite(pop.p16.float()).all().item(), "p32 finite:",
          torch.isfinite(pop.p32).all().item())
    e = ops.embedding(tok.reshape(-1), W["embed"], rpt)
    rep("embed", e, ops.embed_ref(tok.reshape(-1), W["embed"], rpt))
    h = ops.rmsnorm(e, W["l0.attn_norm"], rpt)
    rep("rmsnorm", h, ops.rmsnorm_ref(e, W["l0.attn_norm"], rpt))
    qkv = torch.bmm(h.view(P, rpt, d), W["l0.wqkv"]).view(R, 3 * d)
    rep("qkv", qkv, torch.bmm(h.float().view(P, rpt, d), W["l0.wqkv"].float()).view(R, 3 * d))
    q, k, v = ops.rope_split(qkv, pop.cos, pop.sin, T, H)
    qr, kr, vr = ops.rope_split_ref(qkv, pop.cos, pop.sin, T, H)
    rep("q", q, qr)
    rep("k", k, kr)
    rep("v", v, vr)
    o = ops.attention(q, k, v)
    rep("attn", o, ops.attention_ref(q, k, v, 0.125))
    gu = torch.bmm(h.view(P, rpt, d), W["l0.wgu"])
    a = ops.swiglu(gu)
    rep("swiglu", a, ops.swiglu_ref(gu))
    logits = torch.bmm(h.view(P, rpt, d), W["head"][:, :, :]).reshape(R, c.vocab)
    lab = tgt.reshape(-1)
    rep("ce_eval", ops.ce_eval(logits.clone(), lab, rpt), ops.ce_ref(logits, lab, rpt))
    print("full fwd eval:", pop._forward(tok, tgt, train=False))
loss = pop._forward(tok, tgt, train=True)
print("full fwd train:", loss)
