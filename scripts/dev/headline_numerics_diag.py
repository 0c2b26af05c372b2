"""Where do the HIP and torch-reference populations differ after one step at the headline
shapes?  Per variant (stream groups, population subsets) and slot: max |dm| / max |m| of each
layer's momentum (= the first step's gradient) against the fp32 reference with bf16 emulation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.ops.population import PopulationMLP
from tests.test_headline_numerics_gpu import _configs

data = TeacherClassification(n_train=128 * 64, n_val=1024, batch_size=128, seed=11, device="cuda")
x, y = data.batch(0)
CFGS = _configs()
SLOTS = [2 * i + (i % 2) for i in range(len(CFGS))]


def build(backend, streams, members, cap=32, mw=1024):
    p = PopulationMLP(cap, max_width=mw, n_hidden=3, eval_batch=1024, device="cuda",
                      backend=backend, momentum_dtype="fp32",
                      n_streams=streams if backend == "hip" else None)
    for s, c in members:
        p.set_member(s, c)
    return p


def rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def run(tag, streams, members, **kw):
    hip, ref = build("hip", streams, members, **kw), build("torch", 1, members, **kw)
    hip.train_step(x, y)
    ref.train_step(x, y)
    torch.cuda.synchronize()
    out = []
    for s, c in members:
        errs = [rel(hip.layer_views(s, hip.m32)[l][0].float(), ref.layer_views(s, ref.m32)[l][0].float())
                for l in range(4)]
        out.append(f"{s}:w{c.width}:" + "/".join(f"{e:.3f}" for e in errs))
    print(f"{tag:28s} " + "  ".join(out), flush=True)


allm = list(zip(SLOTS, CFGS))
run("all, 3 streams", 3, allm)
run("all, 1 stream", 1, allm)
bad = [m for m in allm if m[0] in (8, 24, 31, 7)]
run("4 members, 1 stream", 1, bad)
for m in bad:
    run(f"alone slot {m[0]} 1 stream", 1, [m])
    run(f"alone slot 0 1 stream", 1, [(0, m[1])])
    run(f"alone cap1 mw1024", 1, [(0, m[1])], cap=1)
