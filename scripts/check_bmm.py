"""Check population-batched bf16 GEMMs against per-trial fp32 matmuls: the three GEMMs of a
linear layer (y = x w, dx = g w^T, dw = x^T g) in the layouts autograd uses (transposed operand
views) and with the transposes materialised (plain NN GEMMs)."""
import sys

import torch

P, M = 8, 4096
shapes = [(768, 2304), (768, 768), (768, 4096), (2048, 768), (768, 32000), (256, 704),
          (704, 256), (256, 4096)]
for lib in [a for a in sys.argv[1:] if not a.startswith("--")]:
    torch.backends.cuda.preferred_blas_library(lib)
print("== blas", torch.backends.cuda.preferred_blas_library(), flush=True)


def bad(got, ref):
    e = (got.float() - ref).abs().amax((1, 2)) / (ref.abs().amax((1, 2)) + 1e-12)
    return [i for i, v in enumerate(e.tolist()) if not (v < 2e-2)]


for K, N in shapes:
    torch.manual_seed(0)
    x = (torch.randn(P, M, K, device="cuda") * 0.1).to(torch.bfloat16)
    w = (torch.randn(P, K, N, device="cuda") * 0.02).to(torch.bfloat16)
    g = (torch.randn(P, M, N, device="cuda") * 1e-3).to(torch.bfloat16)
    xf, wf, gf = x.float(), w.float(), g.float()
    ref_dx, ref_dw = torch.bmm(gf, wf.transpose(1, 2)), torch.bmm(xf.transpose(1, 2), gf)
    res = {
        "y": bad(torch.bmm(x, w), torch.bmm(xf, wf)),
        "dx_NN": bad(torch.bmm(g, w.transpose(1, 2).contiguous()), ref_dx),
        "dw_NN": bad(torch.bmm(x.transpose(1, 2).contiguous(), g), ref_dw),
        "dx_loop": bad(torch.stack([g[p] @ w[p].t() for p in range(P)]), ref_dx),
    }
    if "--transposed" in sys.argv:   # (K=2048, N=768) dx_T faults in the installed hipBLASLt
        res["dx_T"] = bad(torch.bmm(g, w.transpose(1, 2)), ref_dx)
        res["dw_T"] = bad(torch.bmm(x.transpose(1, 2), g), ref_dw)
    torch.cuda.synchronize()
    print(f"K={K} N={N}: {res}", flush=True)
