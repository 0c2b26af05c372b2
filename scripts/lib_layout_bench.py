"""hipBLASLt (torch.bmm) on the transposed-view layouts the LM backward needs (dX = dY W^T,
dW = X^T dY) vs the population GEMM, with a numerics cross-check.  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.ops.gemm import pgemm  # noqa: E402
from scripts.gemm_bench import SHAPES, timeit  # noqa: E402


def main():
    for name, P, M, N, K, ta, tb in SHAPES:
        if not (ta or tb) or name.startswith("rn."):
            continue
        a = torch.randn(P, K, M, device="cuda").to(torch.bfloat16) if ta else \
            torch.randn(P, M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(P, N, K, device="cuda").to(torch.bfloat16) if tb else \
            torch.randn(P, K, N, device="cuda").to(torch.bfloat16)
        out = torch.empty(P, M, N, device="cuda", dtype=torch.bfloat16)
        out2 = torch.empty_like(out)
        av = a.transpose(1, 2) if ta else a
        bv = b.transpose(1, 2) if tb else b
        flops = 2.0 * P * M * N * K
        t_p = timeit(lambda: pgemm(a, b, ta=ta, tb=tb, out=out), 20)
        t_l = timeit(lambda: torch.bmm(av, bv, out=out2), 20)
        ref = torch.bmm(av.float(), bv.float())
        scale = ref.abs().max().item()
        print(json.dumps({"shape": name, "pgemm_tflops": round(flops / t_p / 1e6, 1),
                          "bmm_view_tflops": round(flops / t_l / 1e6, 1),
                          "pgemm_err": round((out.float() - ref).abs().max().item() / scale, 5),
                          "bmm_err": round((out2.float() - ref).abs().max().item() / scale, 5)}),
              flush=True)


if __name__ == "__main__":
    main()
