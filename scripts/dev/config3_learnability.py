"""Config 3's synthetic task: validation loss of ResNet-20 members over the 390-step trial budget
(lr 0.1 / 0.05 / 0.02 with momentum 0.9, weight decay 5e-4, and an lr-0 control), printed every
65 steps, twice from the same seeds (run-to-run determinism)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from metaopt_amd.models.resnet import PopulationResNet, SyntheticCIFAR
from metaopt_amd.ops.population import MemberConfig

data = SyntheticCIFAR(n_train=390 * 128, n_val=1024, batch_size=128, seed=0, device="cuda")
p = torch.bincount(data.val_y.cpu(), minlength=10).double() / len(data.val_y)
print("H(y)", float(-(p[p > 0] * p[p > 0].log()).sum()), flush=True)
for rep in range(2):
    pop = PopulationResNet(4, batch_size=128, device="cuda", blocks_per_stage=3, image_size=32)
    for s, lr in enumerate((0.1, 0.05, 0.02, 0.0)):
        pop.set_member(s, MemberConfig(width=0, lr=lr, momentum=0.9, weight_decay=5e-4, seed=1 + s))
    for step in range(390):
        pop.train_step(*data.batch(step))
        if (step + 1) % 65 == 0:
            vl, va = pop.evaluate(*data.validation())
            tl = pop.train_loss()
            print(rep, step + 1, "val", [round(float(v), 3) for v in vl],
                  "acc", [round(float(v), 3) for v in va],
                  "train", [round(float(v), 3) for v in tl], flush=True)
