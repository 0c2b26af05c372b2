"""f32-operand population GEMM plans (the K11 second-order step's shapes): time every
(tile cfg, split-K) candidate per shape and print the best against the default plan.

    python scripts/gemm_f32_bench.py [--out FILE]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.ops.gemm import pgemm, plan  # noqa: E402

# (label, P, M, N, K, ta, tb): tiny-2layer, P = 8 runs, R = 512 rows, S = 3 slices
SHAPES = [
    ("qkv.fwd", 8, 1536, 768, 256, False, False),
    ("qkv.tan", 16, 512, 768, 256, False, False),
    ("wgu.fwd", 8, 1536, 1408, 256, False, False),
    ("down.fwd", 8, 1536, 256, 704, False, False),
    ("head.fwd", 8, 1536, 4096, 256, False, False),
    ("head.tan", 16, 512, 4096, 256, False, False),
    ("qkv.dx", 8, 1536, 256, 768, False, True),
    ("head.dx", 8, 1536, 256, 4096, False, True),
    ("wgu.dx", 8, 1536, 256, 1408, False, True),
    ("qkv.dw", 24, 256, 768, 512, True, False),
    ("wgu.dw", 24, 256, 1408, 512, True, False),
    ("down.dw", 24, 704, 256, 512, True, False),
    ("head.dw", 24, 256, 4096, 512, True, False),
    ("attn.s", 128, 384, 128, 64, False, True),
    ("attn.pv", 128, 384, 64, 128, False, False),
    ("attn.dk", 384, 128, 64, 128, True, False),
]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    res = []
    for label, P, M, N, K, ta, tb in SHAPES:
        a = torch.randn(P, *((K, M) if ta else (M, K)), device=dev)
        b = torch.randn(P, *((N, K) if tb else (K, N)), device=dev)
        out = torch.empty(P, M, N, device=dev)
        flop = 2.0 * P * M * N * K
        default = plan(P, M, N, K)
        dflt = bench(lambda: pgemm(a, b, ta=ta, tb=tb, out=out))
        cands = {}
        for cfg in (0, 2, 3, 4):
            for sp in (1, 2, 4):
                if sp > 1 and K // sp < 128:
                    continue
                try:
                    cands[(cfg, sp)] = bench(lambda: pgemm(a, b, ta=ta, tb=tb, out=out, cfg=cfg,
                                                           splits=sp))
                except Exception as ex:                                  # noqa: BLE001
                    print(label, cfg, sp, ex)
        best = min(cands, key=cands.get)
        rec = dict(shape=label, P=P, M=M, N=N, K=K, ta=ta, tb=tb, default_plan=list(default),
                   default_us=round(dflt, 2), best=list(best), best_us=round(cands[best], 2),
                   default_tflops=round(flop / dflt / 1e6, 1),
                   best_tflops=round(flop / cands[best] / 1e6, 1),
                   all={f"{c}/{s}": round(v, 2) for (c, s), v in cands.items()})
        res.append(rec)
        print(json.dumps(rec), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
