"""Which Python call sites launch the small framework kernels (fills, casts, copies) of the
population ResNet-20 train step: torch.profiler with stacks over a few steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from metaopt_amd.worker.tasks import get  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    spec = get("resnet20")
    task, pop, data = spec.build(32, dev, 0, steps_per_trial=390)
    for s in range(pop.capacity):
        pop.set_member(s, task.member_config({"/lr": 0.05, "/momentum": 0.9,
                                              "/weight_decay": 5e-4}, s + 1))
    for i in range(3):
        pop.train_step(*data.batch(i))
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as p:
        for i in range(3, 6):
            pop.train_step(*data.batch(i))
        torch.cuda.synchronize()
    tab = p.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=40,
                                                     max_name_column_width=60)
    print(tab)


if __name__ == "__main__":
    main()
