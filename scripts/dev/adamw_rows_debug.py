"""Per-layer HIP-vs-reference deviation of AdamW members with 1..3 row blocks (debug aid):
fraction of weights off by more than lr/2 after a few steps."""
import torch

from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.ops.population import MemberConfig, PopulationMLP

data = TeacherClassification(n_train=384 * 12, n_val=256, batch_size=384, seed=5, device="cuda")
for pop_rows in (128, 384):
    cfgs = [MemberConfig(width=256, lr=0.002, momentum=m, weight_decay=5e-4, dropout=d,
                         seed=23 + i, batch_size=b)
            for i, (b, m, d) in enumerate([(128, 0.0, 0.1), (128, 0.9, 0.1), (128, 0.0, 0.0),
                                           (384, 0.0, 0.1), (384, 0.9, 0.1), (384, 0.0, 0.0)])
            if b <= pop_rows]
    for steps in (1, 2, 3):
        pops = []
        for backend in ("hip", "torch"):
            p = PopulationMLP(8, max_width=256, batch_size=pop_rows, eval_batch=256,
                              optimizer="adamw", device="cuda", backend=backend)
            for i, c in enumerate(cfgs):
                p.set_member(i + 1, c)
            pops.append(p)
        for step in range(steps):
            x, y = data.batch(step)
            for p in pops:
                p.train_step(x[:pop_rows], y[:pop_rows])
        torch.cuda.synchronize()
        hip, ref = pops
        for s in ref.active_slots():
            c = cfgs[s - 1]
            out = []
            for l, ((wh, _), (wr, _)) in enumerate(zip(hip.layer_views(s), ref.layer_views(s))):
                d = (wh - wr).abs()
                out.append(f"L{l} {float((d > c.lr / 2).float().mean()):.2e}")
            print(f"pop {pop_rows} steps {steps} rows {c.batch_size} b1 {c.momentum} "
                  f"drop {c.dropout}: " + " ".join(out), flush=True)
