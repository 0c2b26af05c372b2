"""Throughput of the population GEMM kernel (csrc/pgemm.hip) vs torch.bmm (hipBLASLt) on the
GEMM shapes of the 125M LM (8 trials x 4096 tokens) and ResNet-20 (32 trials), in every layout
the training step uses.  Prints one line per shape and a JSON summary (--out)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.ops.gemm import MF32_TILES, pgemm, plan  # noqa: E402

# (name, P, M, N, K, ta, tb)
SHAPES = [
    ("lm.qkv.fwd", 8, 4096, 2304, 768, False, False),
    ("lm.qkv.dx", 8, 4096, 768, 2304, False, True),
    ("lm.qkv.dw", 8, 768, 2304, 4096, True, False),
    ("lm.wo.fwd", 8, 4096, 768, 768, False, False),
    ("lm.wo.dx", 8, 4096, 768, 768, False, True),
    ("lm.wo.dw", 8, 768, 768, 4096, True, False),
    ("lm.gu.fwd", 8, 4096, 4096, 768, False, False),
    ("lm.gu.dx", 8, 4096, 768, 4096, False, True),
    ("lm.gu.dw", 8, 768, 4096, 4096, True, False),
    ("lm.down.fwd", 8, 4096, 768, 2048, False, False),
    ("lm.down.dx", 8, 4096, 2048, 768, False, True),
    ("lm.down.dw", 8, 2048, 768, 4096, True, False),
    ("lm.head.fwd", 8, 4096, 32000, 768, False, False),
    ("lm.head.dx", 8, 4096, 768, 32000, False, True),
    ("lm.head.dw", 8, 768, 32000, 4096, True, False),
    ("rn.s1.fwd", 32, 131072, 16, 144, False, False),
    ("rn.s1.dx", 32, 131072, 144, 16, False, True),
    ("rn.s1.dw", 32, 144, 16, 131072, True, False),
    ("rn.s3.fwd", 32, 8192, 64, 576, False, False),
    ("rn.s3.dw", 32, 576, 64, 8192, True, False),
    # square references: the ceiling of this kernel and of the library away from the LM's short
    # K / narrow N (round 6)
    ("sq.8192", 1, 8192, 8192, 8192, False, False),
    ("sq.p8.4096", 8, 4096, 4096, 4096, False, False),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--cfgs", default="", help="comma-separated tile configs to time as well")
    ap.add_argument("--shapes", default="", help="only shapes whose name starts with this")
    ap.add_argument("--splits", default="", help="cfg:splits pairs to time, e.g. 5:2,5:4,6:2")
    args = ap.parse_args()
    rows = []
    for name, P, M, N, K, ta, tb in SHAPES:
        if not name.startswith(args.shapes):
            continue
        a = torch.randn(P, K, M, device="cuda").to(torch.bfloat16) if ta else \
            torch.randn(P, M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(P, N, K, device="cuda").to(torch.bfloat16) if tb else \
            torch.randn(P, K, N, device="cuda").to(torch.bfloat16)
        out = torch.empty(P, M, N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * P * M * N * K
        t_ours = timeit(lambda: pgemm(a, b, ta=ta, tb=tb, out=out), args.iters)
        row = {"shape": name, "P": P, "M": M, "N": N, "K": K, "plan": plan(P, M, N, K),
               "pgemm_us": round(t_ours, 1), "pgemm_tflops": round(flops / t_ours / 1e6, 1)}
        for c in [int(v) for v in args.cfgs.split(",") if v]:
            if c in MF32_TILES and (ta or not tb):
                continue                          # the 32x32x16 kernel is NT only
            t = timeit(lambda: pgemm(a, b, ta=ta, tb=tb, out=out, cfg=c), args.iters)
            row[f"cfg{c}_tflops"] = round(flops / t / 1e6, 1)
        for pair in [v for v in args.splits.split(",") if v]:
            c, sp = (int(x) for x in pair.split(":"))
            if K % (64 * sp) == 0 and plan(P, M, N, K, c, sp)[:2] == (c, sp):
                t = timeit(lambda: pgemm(a, b, ta=ta, tb=tb, out=out, cfg=c, splits=sp),
                           args.iters)
                row[f"cfg{c}s{sp}_tflops"] = round(flops / t / 1e6, 1)
        if not args.no_torch and not (ta and tb):
            aa = a.transpose(1, 2) if ta else a
            bb = b.transpose(1, 2) if tb else b
            # the library on materialised (contiguous) operands -- its transposed-view forms are
            # the ones that misbehave on this stack
            ac, bc = aa.contiguous(), bb.contiguous()
            t_lib = timeit(lambda: torch.bmm(ac, bc, out=out), args.iters)
            row["bmm_nn_us"] = round(t_lib, 1)
            row["bmm_nn_tflops"] = round(flops / t_lib / 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
