"""Per-kernel time of the LM attention (csrc/lm_attn.hip) at the 125M config's shape: 8 trials x
8 sequences x 12 heads, T = 512, head dim 64.  Forward and backward are timed separately with HIP
events; ``MOPT_KERNEL_LIB`` selects a variant build (occupancy sweeps:
``python -m metaopt_amd.ops.build --variant w243 -D MOPT_ATTN_WAVES=2,4,3``).

    python scripts/attn_bench.py [--iters 20] [--out profiles/x.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.ops import lm as ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bp", type=int, default=64)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--T", type=int, default=512)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.manual_seed(0)
    q, k, v = (torch.randn(a.bp, a.heads, a.T, 64, device="cuda").to(torch.bfloat16)
               .requires_grad_(True) for _ in range(3))
    do = torch.randn(a.bp * a.T, a.heads * 64, device="cuda").to(torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd = bwd = 0.0
    for it in range(a.iters + 3):
        torch.cuda.synchronize()
        ev[0].record()
        o = ops.attention(q, k, v)
        ev[1].record()
        o.backward(do)
        ev[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            fwd += ev[0].elapsed_time(ev[1])
            bwd += ev[1].elapsed_time(ev[2])
        q.grad = k.grad = v.grad = None
    res = {"lib": os.environ.get("MOPT_KERNEL_LIB", "default"),
           "fwd_us": round(1e3 * fwd / a.iters, 1), "bwd_us": round(1e3 * bwd / a.iters, 1)}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
