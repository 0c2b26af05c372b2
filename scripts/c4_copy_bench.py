"""Device-side cost of moving one config-5 member (Llama-style 125M, AdamW, bf16 first moment)
between a slot and the checkpoint pool, on one GPU (VERDICT r3 "C4 for config 5"):

* save  -- slot -> pool (PopulationSweep._apply checkpointing a member that leaves its slot);
* load  -- pool -> slot (a resume or PBT exploit on the same GPU; also what the receiving rank
           of a direct C4 transfer runs after the pool entry arrived);
* pack  -- the round-3 C4 path's extra copies: pack_state on the sender (torch.cat of the pool
           entry) and unpack + load_slot_state on the receiver, which the direct path removes;
* copy_member -- a PBT exploit slot -> slot without the pool.

Every figure is the mean over ``--iters`` timed repetitions (HIP events), with the bytes moved.
``python scripts/c4_copy_bench.py [--iters 10] [--out profiles/r4/c4_copy.json]``
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from metaopt_amd.models.llama import PopulationLM  # noqa: E402
from metaopt_amd.ops.population import MemberConfig  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    pop = PopulationLM(2, "llama-125m", batch_size=8, seq_len=512, device="cuda",
                       moment_dtype=torch.bfloat16, use_graph=False)
    pop.set_member(0, MemberConfig(width=0, lr=1e-3, seed=1))
    pop.set_member(1, MemberConfig(width=0, lr=1e-3, seed=2))
    pop.alloc_ckpt_pool(2)
    n = pop.n_params
    state_bytes = sum(b[:n].element_size() * n for b in pop._state_bufs()) + 2 * n  # + p16
    metas = pop.save_states([(0, 0)])
    res = {"params_per_member": n, "member_state_bytes": state_bytes}
    res["save_ms"] = timed(lambda: pop.save_states([(0, 1)]), a.iters)
    res["load_ms"] = timed(lambda: pop.load_states([(1, metas[0])]), a.iters)

    def packed():
        buf = pop.pack_state(pop.pool_state(metas[0]))
        pop.load_slot_state(1, pop.unpack_state(buf))
    res["pack_unpack_load_ms"] = timed(packed, a.iters)
    res["copy_member_ms"] = timed(lambda: pop.copy_member(0, 1), a.iters)
    for k in ("save", "load"):
        res[f"{k}_GBps"] = round(2 * state_bytes / (res[f"{k}_ms"] * 1e-3) / 1e9, 1)
    res = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
