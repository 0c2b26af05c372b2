"""Probe: can two RCCL ranks share the box's one GPU?  (If so, the nccl code paths of the sweep
-- C1 all_gather, C5 broadcast, C4 batch_isend_irecv, object collectives -- can be exercised on a
one-GPU box.)  Run: python scripts/dev/rccl_two_ranks_one_gpu.py"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    out = torch.empty(world * 4, device="cuda")
    dist.all_gather_into_tensor(out, t)
    box = [{"rank": rank}]
    dist.broadcast_object_list(box, src=0)
    peer = 1 - rank
    s = torch.full((8,), float(rank), device="cuda")
    r = torch.empty(8, device="cuda")
    for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, s, peer),
                                       dist.P2POp(dist.irecv, r, peer)]):
        req.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {t.tolist()} gather {out.tolist()} obj {box[0]} "
          f"p2p {r[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    port = 29500 + os.getpid() % 1000
    mp.start_processes(worker, args=(2, port), nprocs=2, join=True, start_method="spawn")
    print("OK")
    sys.exit(0)
