"""Quick GPU diagnostics: build, one-step numerics vs reference, and population step timing."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.ops import build  # noqa: E402
from metaopt_amd.ops.population import MemberConfig, PopulationMLP  # noqa: E402
from metaopt_amd.models.data import TeacherClassification  # noqa: E402

print("lib", build.build(verbose=True), flush=True)
dev = "cuda"
d = TeacherClassification(n_train=128 * 64, n_val=256, batch_size=128, seed=3, device=dev)
cfgs = [MemberConfig(width=w, lr=0.1, dropout=dr, seed=i + 1)
        for i, (w, dr) in enumerate([(64, 0.0), (100, 0.2), (256, 0.1)])]
pops = {}
for be in ("hip", "torch"):
    p = PopulationMLP(4, max_width=256, eval_batch=256, device=dev, backend=be)
    for i, c in enumerate(cfgs):
        p.set_member(i + 1, c)
    pops[be] = p
for step in range(3):
    x, y = d.batch(step)
    for be, p in pops.items():
        p.train_step(x, y)
    torch.cuda.synchronize()
    print("step", step, "hip", pops["hip"].train_loss(), "ref", pops["torch"].train_loss(), flush=True)
for s in pops["torch"].active_slots():
    for l, ((wh, bh), (wr, br)) in enumerate(zip(pops["hip"].layer_views(s), pops["torch"].layer_views(s))):
        print(f"slot {s} layer {l} max|dW|={float((wh - wr).abs().max()):.3e} "
              f"max|W|={float(wr.abs().max()):.3e} max|db|={float((bh - br).abs().max()):.3e}")
print("eval hip", pops["hip"].evaluate(*d.validation()))
print("eval ref", pops["torch"].evaluate(*d.validation()))

# ---- timing: 256 trials, widths log-uniform in [64, 1024]
rng = np.random.RandomState(0)
P = 256
pop = PopulationMLP(P, max_width=1024, device=dev, backend="hip")
for s in range(P):
    w = int(np.exp(rng.uniform(np.log(64), np.log(1024))))
    pop.set_member(s, MemberConfig(width=w, lr=float(np.exp(rng.uniform(np.log(1e-3), 0))),
                                   dropout=float(rng.uniform(0, 0.5)), seed=s))
x, y = d.batch(0)
for i in range(5):
    pop.train_step(x, y)
torch.cuda.synchronize()
n = 50
t = time.perf_counter()
for i in range(n):
    pop.train_step(*d.batch(i))
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / n
byts = sum(pop.bytes_per_step(s) for s in range(P))
flops = sum(pop.flops_per_step(s) for s in range(P))
print(f"P={P} step {dt*1e3:.3f} ms  param-bytes {byts/1e9:.2f} GB -> {byts/dt/1e12:.2f} TB/s  "
      f"{flops/dt/1e12:.1f} TFLOP/s  mean width {np.mean([m.width for m in pop.members]):.0f}")
