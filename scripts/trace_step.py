#!/usr/bin/env python
"""Per-kernel in-situ times of the population-MLP train step from a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``): every 2L-kernel step (L forwards incl. the loss
kernel, then L backwards top-down) is located in launch order, and each position's mean
duration plus the idle gaps between consecutive kernels are reported.

    python scripts/trace_step.py gpurun_out/r5g/trace_tn64 [--layers 4]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def kind(name):
    if "mlp_fwd_ce" in name:
        return "ce"
    if "mlp_fwd" in name:
        return "fwd"
    if "mlp_bwd" in name:
        return "bwd"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--layers", type=int, default=4)
    args = ap.parse_args()
    L = args.layers
    pattern = ["fwd"] * (L - 1) + ["ce"] + ["bwd"] * L
    names = [f"fwd{l}" for l in range(L - 1)] + [f"ce{L - 1}"] + \
        [f"bwd{l}" for l in range(L - 1, -1, -1)]
    rows = load(args.path)
    kinds = [kind(n) for _, _, n in rows]
    steps = []
    i = 0
    while i + len(pattern) <= len(rows):
        if kinds[i:i + len(pattern)] == pattern:
            steps.append(rows[i:i + len(pattern)])
            i += len(pattern)
        else:
            i += 1
    if not steps:
        raise SystemExit("no complete train step found in the trace")
    dur = {n: [] for n in names}
    gap = {n: [] for n in names[1:]}
    span = []
    for st in steps:
        for j, (s, e, _) in enumerate(st):
            dur[names[j]].append((e - s) / 1e3)
            if j:
                gap[names[j]].append((s - st[j - 1][1]) / 1e3)
        span.append((st[-1][1] - st[0][0]) / 1e3)
    out = {"steps": len(steps),
           "us_per_kernel": {n: round(statistics.median(v), 2) for n, v in dur.items()},
           "gap_us_before": {n: round(statistics.median(v), 2) for n, v in gap.items()},
           "step_span_us_median": round(statistics.median(span), 1),
           "kernel_sum_us": round(sum(statistics.median(v) for v in dur.values()), 1),
           "gap_sum_us": round(sum(statistics.median(v) for v in gap.values()), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
