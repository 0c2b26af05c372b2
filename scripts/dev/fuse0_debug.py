"""Where do the fused-first-layer and separate launches differ?  (debug helper, GPU)"""
import numpy as np
import torch

from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.ops.population import MemberConfig, PopulationMLP

data = TeacherClassification(n_train=128 * 40, n_val=256, batch_size=128, seed=3, device="cuda")
cfgs = [MemberConfig(width=64, lr=0.1, momentum=0.9, weight_decay=1e-4, dropout=0.0, seed=11),
        MemberConfig(width=100, lr=0.05, momentum=0.5, weight_decay=0.0, dropout=0.25, seed=12)]
for mdt in ("fp32", "bf16"):
    for nsteps in (2, 3):
        pops = []
        for fuse in (False, True):
            p = PopulationMLP(3, max_width=256, n_hidden=3, eval_batch=256, device="cuda",
                              backend="hip", n_streams=1, momentum_dtype=mdt)
            p.fuse_first_layer = fuse
            for i, c in enumerate(cfgs):
                p.set_member(i + 1, c)
            pops.append(p)
        batches = [data.batch(k) for k in range(nsteps)]
        for p in pops:
            p.train_steps(batches)
        torch.cuda.synchronize()
        a, b = pops
        print(mdt, nsteps, "loss", a.train_loss()[1:3], b.train_loss()[1:3])
        for s in (1, 2):
            for li, ((wa, ba), (wb, bb)) in enumerate(zip(a.layer_views(s), b.layer_views(s))):
                dw = (wa.float() - wb.float()).abs()
                db = (ba.float() - bb.float()).abs()
                print(f"  slot {s} layer {li}: W diff max {dw.max().item():.3g} n {int((dw > 0).sum())}"
                      f"/{dw.numel()}  b diff max {db.max().item():.3g} n {int((db > 0).sum())}")
            for li, ((ma, _), (mb, _)) in enumerate(zip(a.layer_views(s, a.m32), b.layer_views(s, b.m32))):
                d = (ma.float() - mb.float()).abs()
                print(f"  slot {s} layer {li}: M diff max {d.max().item():.3g} n {int((d > 0).sum())}")
        # act of layer 0 (next-step forward output) after the call
        print("  act equal", torch.equal(a.act, b.act), "grad equal", torch.equal(a.grad, b.grad))
