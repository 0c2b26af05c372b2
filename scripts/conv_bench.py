"""Per-shape timing of the population ResNet convolution kernels (config 3: 32 trials x 128
CIFAR images): forward (+ BN sums), data gradient and weight gradient of every ResNet-20 conv
shape, direct kernels (csrc/conv_direct.hip) vs the implicit GEMM (csrc/pgemm.hip), with the
HBM bytes each must move and the achieved TB/s.

    python scripts/conv_bench.py [--iters 20] [--only fwd|dgrad|wgrad] [--out x.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from metaopt_amd.ops import conv as cops

SHAPES = [  # (stride, Ci, Co, H)
    (1, 8, 16, 32), (1, 16, 16, 32), (2, 16, 32, 32), (1, 32, 32, 16), (2, 32, 64, 16),
    (1, 64, 64, 8)]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--P", type=int, default=32)
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--only", default=None)
    ap.add_argument("--implicit", action="store_true", help="also time the implicit GEMM")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    P, B, dev = a.P, a.B, "cuda"
    rows = []
    for stride, Ci, Co, H in SHAPES:
        OH = H // stride
        x = torch.randn(P * B, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (0.1 * torch.randn(P, 9 * Ci, Co, device=dev)).to(torch.bfloat16)
        y = torch.empty(P * B, OH, OH, Co, dtype=torch.bfloat16, device=dev)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        sums = torch.zeros(P, 2, Co, device=dev)
        bx, by = x.numel() * 2, y.numel() * 2
        jobs = {"fwd": (0, x, w, y, sums, bx + by), "dgrad": (1, dy, w, dx, None, bx + by),
                "wgrad": (2, x, dy, dw, None, bx + by)}
        for kind, (k, A, Bm, out, s, nbytes) in jobs.items():
            if a.only and kind != a.only:
                continue
            if kind == "dgrad" and Ci == 8:
                continue
            r = {"shape": f"s{stride} {Ci}->{Co} @{H}", "kind": kind, "MB": round(nbytes / 1e6, 1)}
            cops._DIRECT = True
            us = timed(lambda: cops._pconv(k, A, Bm, out, P, B, H, H, Ci, Co, stride, s), a.iters)
            r["direct_us"] = round(us, 1)
            r["direct_TBps"] = round(nbytes / us / 1e6, 2)
            if a.implicit:
                cops._DIRECT = False
                us = timed(lambda: cops._pconv(k, A, Bm, out, P, B, H, H, Ci, Co, stride),
                           a.iters)
                r["implicit_us"] = round(us, 1)
                cops._DIRECT = True
            rows.append(r)
            print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
