"""Per-kernel timing of one population step (256 members, widths ~ loguniform(64, 1024)).

Reports time per launch (HIP events) and effective bandwidth against the per-parameter byte
model of each kernel (fwd: 2 B/param bf16 weight read; bwd+SGD: 16 B/param, 12 with the bf16
momentum buffer -- split f32 master read and written as hi/lo halves).
"""
import os
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.models.data import TeacherClassification  # noqa: E402
from metaopt_amd.ops import _lib  # noqa: E402
from metaopt_amd.ops.population import (BWD_HAS_DX, BWD_IN_DROPOUT, BWD_NARROW, BWD_UPDATE_BIAS,  FWD_NARROW_CE, NARROW_CLASSES,  # noqa: E402
                                        FWD_DROPOUT, FWD_RELU, FWD_WRITE_GRAD, MemberConfig,
                                        PopulationMLP)

ap = argparse.ArgumentParser()
ap.add_argument("--population", type=int, default=256)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--width", type=int, default=0, help="fixed width (0: loguniform(64,1024))")
ap.add_argument("--optimizer", default="sgd")
ap.add_argument("--momentum-dtype", default="fp32", choices=["fp32", "bf16"])
ap.add_argument("--streams", type=int, default=1)
ap.add_argument("--batch", type=int, default=128, help="rows per step (multiple of 128)")
ap.add_argument("--out", default="")
args = ap.parse_args()

dev = torch.device("cuda")
rng = np.random.RandomState(0)
P = args.population
B, RB = args.batch, args.batch // 128
pop = PopulationMLP(P, max_width=1024, device=dev, optimizer=args.optimizer, batch_size=B,
                    momentum_dtype=args.momentum_dtype, n_streams=args.streams)
for s in range(P):
    w = args.width or int(np.exp(rng.uniform(np.log(64), np.log(1024))))
    pop.set_member(s, MemberConfig(width=w, lr=0.01, dropout=0.1, seed=s))
data = TeacherClassification(n_train=B * 8, n_val=128, batch_size=B, seed=0, device=dev)
x, y = data.batch(0)
for _ in range(5):
    pop.train_step(x, y)
torch.cuda.synchronize()

lib, tb, L = pop._lib, pop._tables["train"], pop.L
stream = _lib.stream_ptr(dev)
opt = (2 if args.momentum_dtype == "bf16" else 0) if args.optimizer == "sgd" else 1
BWD_BYTES = {0: 16, 1: 24, 2: 12}[opt]
_narrow = pop.num_classes <= NARROW_CLASSES and os.environ.get("MOPT_NARROW", "1") == "1"
NARROW_CE, NARROW_BWD = (FWD_NARROW_CE, BWD_NARROW) if _narrow else (0, 0)     # split master r+w 8, + momentum (+ AdamW v)


def run_fwd(l):
    src = x if l == 0 else pop.act
    if l < L - 1:
        lib.mopt_mlp_fwd(tb["tl"].data_ptr(), tb["fwd"][l].data_ptr(), tb["n_fwd"][l], RB,
                         src.data_ptr(), pop.plo.data_ptr(), pop.p16.data_ptr(),
                         pop.act.data_ptr(), pop.hp_dev.data_ptr(), 0, l, FWD_RELU | FWD_DROPOUT,
                         pop.fwd_tn, stream)
    else:
        lib.mopt_mlp_fwd_ce(tb["tl"].data_ptr(), tb["fwd"][l].data_ptr(), tb["n_fwd"][l], RB,
                            src.data_ptr(), pop.plo.data_ptr(), pop.p16.data_ptr(), y.data_ptr(),
                            pop.grad.data_ptr(), pop.loss.data_ptr(), pop.correct.data_ptr(),
                            pop.hp_dev.data_ptr(), -1.0, FWD_WRITE_GRAD | NARROW_CE, stream)


def run_bwd(l):
    src = x if l == 0 else pop.act
    flags = BWD_UPDATE_BIAS | ((BWD_HAS_DX | BWD_IN_DROPOUT) if l > 0 else 0) | \
        (NARROW_BWD if l == L - 1 else 0)
    lib.mopt_mlp_bwd(tb["tl"].data_ptr(), tb["bwd"][l].data_ptr(), tb["n_bwd"][l], src.data_ptr(),
                     pop.grad.data_ptr(), pop.plo.data_ptr(), pop.p16.data_ptr(),
                     pop.m32.data_ptr(), pop.v32.data_ptr(), pop.hp_dev.data_ptr(), opt, flags,
                     pop.batch_size // 128, stream)


tl = tb["tl_np"]
layer_params = []
for l in range(L):
    rows = tl[np.array([s * L + l for s in pop.active_slots()])]
    layer_params.append(int((rows["K"].astype(np.int64) * rows["N"]).sum()))

results = {}
for name, fn, byte_per in [("fwd", run_fwd, 2), ("bwd", run_bwd, BWD_BYTES)]:
    for l in range(L):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(args.iters):
            fn(l)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / args.iters
        n = tb["n_fwd"][l] if name == "fwd" else tb["n_bwd"][l]
        gbps = layer_params[l] * byte_per / (ms * 1e-3) / 1e9
        flops = 2 * B * layer_params[l] * (1 if name == "fwd" else (2 if l > 0 else 1))
        results[f"{name}{l}"] = dict(ms=round(ms, 4), workgroups=n, params=layer_params[l],
                                     GBps=round(gbps, 1), TFLOPs=round(flops / ms / 1e9, 1))
        print(f"{name}{l}: {ms*1e3:8.1f} us  WG={n:6d}  params={layer_params[l]/1e6:7.2f}M "
              f"-> {gbps:7.1f} GB/s (param bytes)  {flops/ms/1e9:6.1f} TFLOP/s", flush=True)
if pop.fuse_first_layer and RB == 1 and L >= 2 and len(pop._parts) == 1:
    # the fused first layer (backward + update of step t, forward of step t + 1): one pass over W0
    x2, _ = data.batch(1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):
        _lib.check(lib.mopt_mlp_bwd0_fwd(pop._parts[0]["step_ptr"], x.data_ptr(), x2.data_ptr(),
                                         stream), "mlp_bwd0_fwd")
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / args.iters
    gbps = layer_params[0] * (BWD_BYTES + 0) / (ms * 1e-3) / 1e9
    results["bwd0f"] = dict(ms=round(ms, 4), workgroups=pop._parts[0]["n_bwd0f"],
                            params=layer_params[0], GBps=round(gbps, 1))
    print(f"bwd0f: {ms*1e3:8.1f} us  WG={pop._parts[0]['n_bwd0f']:6d}  (bwd0 + next fwd0, "
          f"{gbps:7.1f} GB/s of backward param bytes)", flush=True)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(args.iters):
    pop.train_step(x, y)
ev1.record()
torch.cuda.synchronize()
step = ev0.elapsed_time(ev1) / args.iters
total_params = sum(layer_params)
print(f"full step: {step*1e3:.1f} us; params {total_params/1e6:.1f}M; "
      f"{total_params*(2 + BWD_BYTES)/(step*1e-3)/1e12:.2f} TB/s param-bytes")
results["step_ms"] = step
if args.out:
    with open(args.out, "w") as f:
        json.dump(results, f, indent=1)
